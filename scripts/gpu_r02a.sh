#!/bin/bash
# Round-2 GPU step A: new-component GPU tests (foot placement, WBIC QP), ABI latency probe,
# then the counter passes of scripts/gpu_pmc_all.sh. Each step has its own limit; stops at the
# first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02a
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 5 60 quad-periodic-mpc_amd/cmpc_abi_latency 10 200 > "$OUT/abi10.txt" 2>&1
echo "abi10 rc=$?"; tail -2 "$OUT/abi10.txt"
timeout -k 10 600 python -u -m pytest tests/test_quadprog.py tests/test_assemble.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_new.log" 2>&1
rc=$?; echo "pytest_new rc=$rc"; tail -15 "$OUT/pytest_new.log"
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_pmc_all.sh r02_pmc1 cfg3 cfg5
