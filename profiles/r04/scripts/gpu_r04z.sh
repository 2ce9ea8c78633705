#!/bin/bash
# r04: the register-sums A/B (tools/gpu_r04y.sh), then the closing
# measurements on build (tools/gpu_r04s.sh: whole suite, profile set,
# logical shards).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r04y timeout -k 10 450 bash tools/gpu_r04y.sh || { echo "A/B failed"; exit 1; }
TAG=r04x timeout -k 10 900 bash tools/gpu_r04s.sh
