#!/bin/bash
# GPU validation session: smoke, then the GPU tests (all, no -x), each under its own time limit.
# usage: scripts/gpu_tests.sh <tag> [pytest selection ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-tests}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
SEL=${*:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest.log | tail -30
sed -n '/parity ledger/,$p' $OUT/pytest.log | head -60
exit $rc
