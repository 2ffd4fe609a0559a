#!/bin/bash
# round-5 GPU call 33: the whole GPU suite and smoke on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05zj GATHER=0 BENCH=0 bash tools/r05_check.sh
