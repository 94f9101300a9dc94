#!/bin/bash
# Class-1 wave placement / latency by batch size (CMPC_PLACE_PROF variant), and the same with
# extra dynamic LDS limiting class-1 workgroups per CU. Each step time-limited; stops at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-place}
mkdir -p "$OUT"
export TMPDIR=/tmp CMPC_LIB=$PWD/variants/libplace.so
step() { local name=$1; local t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 12 | cut -c1-420; return $rc; }
step place_default 300 python3 -u scripts/place_prof.py --batches 64,256,1024,4096,16384,65536 || exit 1
step place_dyn30k 300 env CMPC_C1_DYN_LDS=30000 python3 -u scripts/place_prof.py --batches 256,1024,4096,16384 || exit 1
step place_dyn140k 300 env CMPC_C1_DYN_LDS=140000 python3 -u scripts/place_prof.py --batches 256,1024 || exit 1
step place_mix 300 python3 -u scripts/place_prof.py --batches 4096,65536 --random-contact-frac 0.25 || exit 1
