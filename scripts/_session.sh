set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05_m; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python3 -u scripts/stream_probe.py > $OUT/probe.log 2>&1 || { tail -5 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
CMPC_LIB=variants/knobs.so CMPC_T8_POS=1 timeout -k 10 200 python3 -u scripts/stream_probe.py > $OUT/probe_p1.log 2>&1 || { tail -5 $OUT/probe_p1.log; exit 1; }
echo "--- t8 behind class 1"; cat $OUT/probe_p1.log
CMPC_LIB=variants/knobs.so CMPC_TAIL=0 timeout -k 10 200 python3 -u scripts/stream_probe.py > $OUT/probe_nt.log 2>&1 || { tail -5 $OUT/probe_nt.log; exit 1; }
echo "--- no tail"; cat $OUT/probe_nt.log
