#!/bin/bash
# N = 20 trot phase split of the w120 class (n = 120 trot): default library vs diagnostic variants that stop
# after the Cholesky (diag1), after J = L^-T (diag2) and after the condensation (diag3). Timing only (results of the variants
# are not solutions).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in default variants/libdiag2.so variants/libdiag1.so variants/libdiag3.so; do
  if [ "$v" = default ]; then unset CMPC_LIB; else export CMPC_LIB=$PWD/$v; fi
  echo "== $v"
  timeout -k 10 200 python -u bench.py --horizon 20 --random-contact-frac 0 --steps 5 --warmup 2 --no-cpu-baseline --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][0]); print(d['ms_per_step'], d['roofline']['tail_avg_ms'])" || exit 1
done
