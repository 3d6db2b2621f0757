"""CPU (gloo, world_size 2): instance sharding and the scatter/gather of cmpc.dist."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cmpc import dist as cdist


def test_shard_bounds_partition():
    for B in (0, 1, 7, 64, 65536):
        for W in (1, 2, 3, 8):
            spans = [cdist.shard_bounds(B, r, W) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(spans[r][1] == spans[r + 1][0] for r in range(W - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, N, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cmpc import synth
        full = synth.make_config(2, B=B)
        batch = None
        if rank == 0:
            batch = {k: torch.as_tensor(full[k], dtype=torch.uint8 if k == "contact" else torch.float32)
                     for k in cdist.FIELDS}
        mine = cdist.scatter_batch(batch, B, N, "cpu")
        lo, hi = cdist.shard_bounds(B, rank, world)
        ok = all(np.allclose(mine[k].numpy(), full[k][lo:hi].astype(mine[k].numpy().dtype))
                 for k in cdist.FIELDS)
        # stand-in "solution": a deterministic function of the instance's own inputs
        w = torch.cat([mine["x0"], mine["Bd"].reshape(hi - lo, -1)[:, :24 * N - 12]], 1)
        g = cdist.gather_solutions(w, B)
        if rank == 0:
            ref = np.concatenate([full["x0"], full["Bd"].reshape(B, -1)[:, :24 * N - 12]], 1)
            ok = ok and np.allclose(g.numpy(), ref.astype(np.float32))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [5, 64])
def test_scatter_gather_gloo_world2(B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, 16, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_bench_spawns_ranks_and_shards_config3():
    """`python bench.py --gpus 2` relaunches itself under torch.distributed.run with 2 ranks
    (before any GPU call); with the solve stubbed (CMPC_BENCH_DRYRUN=1, gloo) both ranks report,
    their contiguous slices tile the 65,536-instance config-3 batch, and the timing is the
    max over ranks of the barrier-bracketed region."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    env = dict(os.environ, CMPC_BENCH_DRYRUN="1")
    r = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["ranks_reporting"] == 2
    assert line["spans"] == [[0, 32768], [32768, 65536]]
    assert line["solved_per_step"] == 65536 and line["stub_work"] == 65536 * 4
    assert line["steps"] == 3 and line["warmup"] == 1


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    env = dict(os.environ, CMPC_BENCH_DRYRUN="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
