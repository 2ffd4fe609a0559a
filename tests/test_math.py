"""The fp32 math contract (oracle/glsl_math.h == csrc/pt_math.h).

CPU tests pin the oracle's transcendentals to libm (double precision) within
a few ulp and its RNG to an independent numpy restatement of
raytrace_comp.comp:209-216.  The GPU test checks the device build of the same
functions is bitwise identical to the oracle on millions of inputs.
"""
import numpy as np
import pytest

import oracle_lib as O

FN = {"log": 0, "exp": 1, "sin": 2, "cos": 3, "tan": 4, "acos": 5, "sqrt": 6, "rng": 7, "rcp": 8}


def _ulp_err(got, want64):
    got = got.astype(np.float64)
    want32 = want64.astype(np.float32)
    ulp = np.abs(np.spacing(want32).astype(np.float64))
    ok = np.isfinite(want64)
    return np.max(np.abs(got[ok] - want64[ok]) / ulp[ok])


def _domain(name, n=200000, seed=0):
    rng = np.random.default_rng(seed)
    if name == "log":
        x = np.exp(rng.uniform(np.log(1e-38), 0.0, n)).astype(np.float32)
        x = np.concatenate([x, np.float32([1e-38, 1.0, 0.5, 2.0, 1.17549435e-38, 3e-39])])
    elif name == "exp":
        x = rng.uniform(-100, 10, n).astype(np.float32)
    elif name in ("sin", "cos"):
        x = np.concatenate([rng.uniform(0, 2 * np.pi, n), rng.uniform(-20, 20, n // 4)]).astype(np.float32)
        x = np.concatenate([x, np.float32([0.0, 6.2831855, np.pi / 2, np.pi, 1e-8])])
    elif name == "tan":
        x = rng.uniform(0, 1.4, n).astype(np.float32)
    elif name == "acos":
        x = np.concatenate([rng.uniform(-1, 1, n), rng.uniform(0.99, 1.0, n // 4)]).astype(np.float32)
        x = np.concatenate([x, np.float32([-1.0, 1.0, 0.0, 0.5, -0.5, 1e-9])])
    else:
        x = rng.uniform(0, 4, n).astype(np.float32)
    return x


@pytest.mark.parametrize("name,ref,max_ulp", [
    ("log", np.log, 2.0), ("exp", np.exp, 2.0), ("sin", np.sin, 2.0), ("cos", np.cos, 2.0),
    ("tan", np.tan, 4.0), ("acos", np.arccos, 2.0), ("sqrt", np.sqrt, 0.5)])
def test_oracle_math_close_to_libm(name, ref, max_ulp):
    x = _domain(name)
    got = O.math(FN[name], x)
    err = _ulp_err(got, ref(x.astype(np.float64)))
    assert err <= max_ulp, f"{name}: {err} ulp"


def test_oracle_math_special_values():
    assert O.math(FN["log"], np.float32([0.0]))[0] == -np.inf
    assert np.isnan(O.math(FN["log"], np.float32([-1.0]))[0])
    assert O.math(FN["exp"], np.float32([-200.0]))[0] == 0.0
    assert O.math(FN["exp"], np.float32([100.0]))[0] == np.inf
    assert O.math(FN["acos"], np.float32([1.0]))[0] == 0.0
    # 1e-38 is subnormal: log must see it, not a flushed zero (raytrace_comp.comp:220)
    assert abs(O.math(FN["log"], np.float32([1e-38]))[0] - np.log(1e-38)) < 1e-4


def _pcg_numpy(seed, n):
    """Independent restatement of stepAndOutputRNGFloat (raytrace_comp.comp:209-216)."""
    s = np.uint32(seed)
    out = []
    with np.errstate(over="ignore"):
        for _ in range(n):
            s = np.uint32(s * np.uint32(747796405) + np.uint32(2891336453))
            r = np.uint32(((s >> ((s >> np.uint32(28)) + np.uint32(4))) ^ s) * np.uint32(277803737))
            r = np.uint32((r >> np.uint32(22)) ^ r)
            out.append(np.float32(r) / np.float32(4294967296.0))
    return np.array(out, np.float32)


@pytest.mark.parametrize("seed", [0, 1, 12345, 2**31 + 7, 2**32 - 1])
def test_rng_matches_independent_restatement(seed):
    assert np.array_equal(O.rng(seed, 64), _pcg_numpy(seed, 64))


def test_rng_can_return_one():
    """float(result)/2^32 rounds to 1.0 for result near 2^32: the shader can
    draw exactly 1.0."""
    assert np.float32(np.uint32(0xFFFFFFFF)) / np.float32(4294967296.0) == np.float32(1.0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["log", "exp", "sin", "cos", "tan", "acos", "sqrt", "rcp"])
def test_device_math_bitwise_equals_oracle(name):
    import ptamd
    x = _domain(name, n=1 << 20, seed=7)
    if name == "rcp":
        x = np.concatenate([x, np.float32([0.0, -0.0, 1e-38, -3e-39, 1e30])])
    dev = ptamd.device_math(FN[name], x)
    ref = O.math(FN[name], x)
    bad = np.flatnonzero(dev.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, f"{name}: {bad.size} mismatches, e.g. x={x[bad[:3]]} dev={dev[bad[:3]]} ref={ref[bad[:3]]}"


@pytest.mark.gpu
def test_device_rng_bitwise_equals_oracle():
    import ptamd
    seeds = np.random.default_rng(3).integers(0, 2**32, 1 << 18, dtype=np.uint64).astype(np.uint32)
    dev = ptamd.device_math(FN["rng"], seeds.view(np.float32))
    ref = np.array([O.rng(int(s), 1)[0] for s in seeds[:2000]], np.float32)
    assert np.array_equal(dev[:2000].view(np.uint32), ref.view(np.uint32))
    ref_all = O.math(FN["rng"], seeds.view(np.float32))
    assert np.array_equal(dev.view(np.uint32), ref_all.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("fn,name", [(0, "rcp"), (1, "log"), (2, "exp"), (3, "acos")])
def test_device_fast_quotients_exhaustive(fn, name):
    """The device evaluates these through rcp/fma quotients instead of IEEE
    division; all 2^32 inputs must give the IEEE definition's bits (pt_math.h)."""
    import ptamd
    bad, first = ptamd.device_math_exhaustive(fn)
    assert bad == 0, f"{name}: {bad} of 2^32 inputs differ, first 0x{first:08x}"
