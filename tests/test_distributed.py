"""CPU, world_size 2 over gloo: the multi-GPU control path of bench.py
(one process per GPU, disjoint batches, barrier + max-over-ranks timing, no
data-path collective)."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench

    r, w, local, dist = bench.init_dist()
    plan = bench.rank_plan("c1", r, 8)
    dist.barrier()
    t = bench.max_over_ranks(dist, 1.0 + r)
    # the per-rank timing rows bench.py gathers (start, end, device span):
    # rank r starts at 100 + r and ends at 110 + 3 r
    rows = bench.gather_rows(dist, [100.0 + r, 110.0 + 3 * r, 7.0 + r])
    span = bench.span_of(rows)
    name, fx = bench.fixture_for("c3", r)
    q.put((r, w, local, t, int(plan.mask[:16].astype(np.uint64).sum()), plan.total, len(plan.segments),
           rows.tolist(), span, name, fx["plan"]["frames"] if fx else None))
    dist.destroy_process_group()


def test_two_ranks_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[0] for o in out] == [0, 1] and all(o[1] == 2 for o in out)
    assert all(o[3] == 2.0 for o in out)              # max over ranks
    assert out[0][4] != out[1][4]                      # disjoint batches (distinct seeds)
    assert out[0][5] == out[1][5] and out[0][6] == 8   # same shape per rank
    # gathered rows identical on both ranks, in rank order
    assert out[0][7] == out[1][7] == [[100.0, 110.0, 7.0], [101.0, 113.0, 8.0]]
    assert out[0][8] == out[1][8] == 13.0              # latest end - earliest start
    # each rank's c3-shaped batch has its own reference fixture
    assert [o[9] for o in out] == ["c5_rank0", "c5_rank1"] and all(o[10] == 1 << 20 for o in out)


def _bench(argv, env_extra=None, timeout=180):
    import subprocess

    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "HVWS_BENCH_DEVICE"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + argv, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_launcher_two_ranks():
    """`bench.py --gpus 2` with no launcher around it starts two rank
    processes itself (RANK / WORLD_SIZE / MASTER_* in their environment, gloo
    rendezvous on 127.0.0.1) and relays rank 0's one JSON line; --dry-run
    stubs the GPU legs, so the plumbing runs here on CPU."""
    import json

    p = _bench(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dry_run"] is True
    pr = out["timing"]["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1]
    # each rank names its card: HIP device index, hipGetDevice, PCI bus id (distinct)
    assert [(r["device"], r["hip_device"]) for r in pr] == [(0, 0), (1, 1)]
    assert [r["pci_bus_id"] for r in pr] == ["0000:01:00.0", "0000:02:00.0"]
    v = out["verified"]["ranks"]
    assert [r["fixture"] for r in v] == ["c5_rank0", "c5_rank1"]
    assert [r["local_rank"] for r in v] == [0, 1] and v[0]["seed"] != v[1]["seed"]
    # each card's own unmask time, fraction of 8 TB/s and of its own ceiling
    for r in pr:
        assert {"unmask_ms_mean", "roofline_frac", "stream_ceiling_GBps", "frac_of_box_ceiling"} <= set(r)
        assert r["roofline_frac"] == round(137.4536e9 / (r["unmask_ms_mean"] * 1e-3) / 1e9 / 8000.0, 4)


def test_bench_per_rank_roofline_shows_a_slow_card():
    """an N-rank line exposes one slow card -- its unmask
    time and HBM fractions arrive through the gloo gather in its own row."""
    import json

    p = _bench(["--gpus", "2", "--dry-run"], {"HVWS_BENCH_DRYRUN_SLOW_RANK": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    pr = out["timing"]["per_rank"]
    assert pr[1]["unmask_ms_mean"] > pr[0]["unmask_ms_mean"] * 1.4
    assert pr[1]["roofline_frac"] < pr[0]["roofline_frac"] and pr[1]["frac_of_box_ceiling"] < pr[0]["frac_of_box_ceiling"]


def test_bench_fixture_per_config():
    """Rank 0's c2 / c4 batch is the one the reference digests were taken of
    (seed 1), c3 ranks take config 5's shards; other ranks of c2 / c4 have none."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.fixture_for("c3", 3)[0] == "c5_rank3"
    assert bench.fixture_for("c2", 0)[0] == "c2" and bench.fixture_for("c4", 0)[0] == "c4"
    assert bench.fixture_for("c2", 1) == (None, None)
    assert bench.rank_seed("c2", 0) == 1 and bench.rank_seed("c3", 0) == 1000


def test_bench_launcher_fails_with_a_rank():
    """A rank that fails makes the launcher exit non-zero (the other rank is
    stopped, no result line is printed)."""
    p = _bench(["--gpus", "2", "--dry-run"], {"HVWS_BENCH_DRYRUN_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_launcher_refuses_too_few_gpus():
    """Fewer visible GPUs than --gpus is an error, never a silent N = 1 run
    (the parent exits before any rank or GPU call)."""
    p = _bench(["--gpus", "4"], {"HIP_VISIBLE_DEVICES": "0"}, timeout=60)
    assert p.returncode == 2 and "refusing" in p.stderr
    assert not p.stdout.strip()


def test_bench_launcher_refuses_ranks_sharing_a_device():
    """Two ranks that report one PCI bus id end the run non-zero with no
    result line: an N-rank line must come from N cards."""
    p = _bench(["--gpus", "2", "--dry-run"], {"HVWS_BENCH_DRYRUN_BUS": "0000:05:00.0"})
    assert p.returncode != 0
    assert "share a device" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bus_id_round_trip():
    sys.path.insert(0, ROOT)
    import bench

    for b in ("0000:05:00.0", "0001:c3:1f.7", "0000:ff:00.1"):
        assert bench.bus_name(bench.bus_number(b)) == b
