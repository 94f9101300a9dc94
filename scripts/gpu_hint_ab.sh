#!/bin/bash
# Round-6 grid hints: the parity tests that exercise them, then a same-box A/B against the
# pre-hint library (variants/old.so) and the hint switched off (CMPC_HINT=0, diagnostic build).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r06_hint3}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "stale or invariance or fast_path or reuse or every_size or hands_off or output_steps" > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/$TAG/pytest.log | tail -12
[ $rc -le 1 ] || exit 1
bash scripts/gpu_lib_env_ab.sh $TAG "4096 32768 65536 262144 n16 cfg5" 2 "variants/old.so|-" "variants/knobs.so|CMPC_HINT=0" "variants/knobs.so|CMPC_HINT=1"
