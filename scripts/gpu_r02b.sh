#!/bin/bash
# Round-2 GPU step B: full GPU test suite + smoke, then counter passes (cfg3, cfg5, n16).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02b
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail "$OUT/smoke.log"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_pmc_all.sh r02_pmc1 cfg3 cfg5 n16
timeout -k 10 300 python -u scripts/split_bench.py > gpurun_out/r02b/split_n10.log 2>&1; tail -12 gpurun_out/r02b/split_n10.log
timeout -k 10 300 python -u scripts/split_bench.py --horizon 20 --random-contact-frac 0 --reps 5 > gpurun_out/r02b/split_n20.log 2>&1; tail -12 gpurun_out/r02b/split_n20.log
