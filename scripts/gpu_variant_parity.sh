#!/bin/bash
# Parity of library variants: the golden / live / deployed-horizon parity tests under each
# CMPC_LIB, printing the pass count and the parity ledger's branch lines.
# usage: scripts/gpu_variant_parity.sh <tag> variants/a.so ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for v in "$@"; do
  n=$(basename "$v" .so)
  CMPC_LIB=$PWD/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "golden or live or deployed" > "$OUT/$n.log" 2>&1
  echo "$n: pytest rc=$? $(grep -E 'passed|failed' "$OUT/$n.log" | tail -1)"
  grep -E "beyond 1e-4 \(cap" "$OUT/$n.log" | sed 's/^/    /'
done
