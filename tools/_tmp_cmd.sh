set -e
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
cd discovering-path-tracer_amd
timeout -k 10 120 ./pt_render ../tests/golden/box.obj -w 1920 -h 1080 -progressive 64 -chunk 8 -orbit-at 24 -cache /tmp/box.ptscene -o /tmp/p.pfm
timeout -k 10 120 ./pt_render ../tests/golden/box.obj -w 1920 -h 1080 -progressive 64 -chunk 1 -cache /tmp/box.ptscene
