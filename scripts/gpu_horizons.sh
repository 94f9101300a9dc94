cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/n20
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/n20/pytest.log 2>&1 || { tail -30 gpurun_out/n20/pytest.log; exit 1; }
tail -1 gpurun_out/n20/pytest.log
for lib in libcmpc_hip.so libcmpc_w128x2.so; do
  for args in "--horizon 20 --random-contact-frac 0" "--horizon 20" "--horizon 16 --random-contact-frac 0"; do
    CMPC_LIB=quad-periodic-mpc_amd/$lib timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 10 $args > gpurun_out/n20/b.log 2>&1 || { tail -5 gpurun_out/n20/b.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/n20/b.log').read().strip().splitlines()[-1]); print('$lib', '$args', d['value'], d['ms_per_step'])"
  done
done
