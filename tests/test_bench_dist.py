"""bench.py's multi-rank path on CPU (gloo, plumbing stand-in for the solve): `--gpus N`
relaunches under torch.distributed.run, config 4 strong-scales the global batch over the ranks
with the root scatter -> solve -> gather pipeline, and the gathered per-instance rows are
bitwise identical to a world-size-1 run (per-instance seeds: every shard holds the instances a
1-GPU run holds)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _bench(*args, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "1",
                        "--warmup", "1", "--no-extras", *args],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus,gb,chunks", [(2, 262144, 4), (3, 10007, 3)])
def test_config4_sharded_equals_single(gpus, gb, chunks):
    one = _bench("--config", "4", "--global-batch", str(gb), "--chunks", str(chunks))
    many = _bench("--gpus", str(gpus), "--global-batch", str(gb), "--chunks", str(chunks))
    assert one["n_gpus"] == 1 and many["n_gpus"] == gpus
    assert many["config"]["config"] == 4 and many["scaling"] == "strong"
    assert one["config"]["global_batch"] == gb and many["config"]["global_batch"] == gb
    assert many["forces_digest"] == one["forces_digest"]
    assert many["status_counts"] == {"ok": gb}


def test_weak_mode_shards_reproduce_ids(cm):
    """Per-rank generation of instance ids [r*B, (r+1)*B) equals slices of one generation."""
    import numpy as np
    full = cm.make_instances(300, 10)
    parts = [cm.make_instances(100, 10, first_id=100 * r) for r in range(3)]
    np.testing.assert_array_equal(np.concatenate(parts), full)
