"""The C-ABI multi-GPU entry point (include/cmpc_multi.h, libcmpc_multi.so) driven by a plain C++
caller (csrc/tools/cmpc_multi_test.cpp, no Python or torch in the solve path): at world 1 and in
the loopback world 2 (the root sends its peer's block of records to itself over RCCL
ncclSend / ncclRecv, a second handle solves it, the forces and status bytes come back the same
way), with the automatic root share, an even split and a 3.5x root share. Every solve must equal a
single cmpc_batch_solve of the whole batch bit for bit (the instances are
independent, so sharding changes nothing)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

EXE = os.path.join(ROOT, "quad-periodic-mpc_amd", "cmpc_multi_test")


@pytest.mark.parametrize("N,B", [(10, 20000), (16, 3000)])
def test_multi_c_abi_bitwise_world1_and_loopback(cm, tmp_path, N, B):
    if not os.path.exists(EXE):
        pytest.fail("cmpc_multi_test not built (quad-periodic-mpc_amd/build.py build_multi)")
    recs = cm.make_instances(B, N, seed=7700 + N, random_contact_frac=0.5)
    f = tmp_path / "recs.f32"
    np.ascontiguousarray(recs, np.float32).tofile(f)
    r = subprocess.run([EXE, str(f), str(B), str(N), "5"], capture_output=True, text=True, timeout=240)
    print(r.stdout, r.stderr[-2000:])
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["all_bitwise"] and len(d["cases"]) == 4
    loop = [c for c in d["cases"] if c["loopback"]]
    assert all(c["rows"][1] > 0 for c in loop)            # a peer block crossed RCCL every time
    assert sum(loop[0]["rows"]) == B and loop[1]["rows"][0] - loop[1]["rows"][1] in (0, 1)
