"""Multi-rank (N>1) path on CPU with the gloo backend.

bench.py shards the record sequence across ranks with no data-path
collective: weak configs seal records [r*n, (r+1)*n) per rank, config 4 splits
ONE fixed batch into contiguous ranges balanced by bytes and config 5 splits
the fixed key set by key ranges; the only collectives are the timing barrier
and max/sum reductions.  These tests run those pieces on gloo ranks: the
per-rank seals (done here by the CPU oracle, the checker) concatenate to
exactly the single-process result, the reductions are max/sum, and
`bench.py --gpus N --plan-only` (the launcher itself: N fresh rank processes,
rendezvous on 127.0.0.1) produces disjoint, covering, byte-balanced shards.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import oracle_lib as o


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _seal_shard(config, first, lens, offs):
    aead, key_len = bench.CONFIGS[config][0], bench.CONFIGS[config][1]
    pt, offs2, nonces, ads = o.synth_batch(first, lens, align=bench.record_align(config))
    assert np.array_equal(offs2, offs)
    keys = np.frombuffer(bench.synth_key(0, key_len), dtype=np.uint8).copy()
    assert bytes(keys) == o.synth_key(0, key_len)
    out = np.zeros_like(pt)
    tags = np.zeros(16 * len(lens), dtype=np.uint8)
    n = len(lens)
    aid = o.AES_GCM if "gcm" in aead else o.CHACHA20_POLY1305
    failed = o.batch(aid, 1, keys, key_len, None, pt, out, offs, lens, nonces, 12, ads,
                     np.arange(n, dtype=np.uint64) * np.uint64(13), np.full(n, 13, np.uint64),
                     tags, 16, threads=2)
    assert failed == 0
    cts = b"".join(out[int(offs[i]):int(offs[i] + lens[i])].tobytes() for i in range(n))
    return hashlib.sha256(cts).hexdigest(), tags.tobytes().hex()


def _worker(rank, world, port, config, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = bench.shard_plan(config, rank, world, records=n)
    first, lens, offs = sh.first, sh.lens, sh.offs
    ct_d, tags = _seal_shard(config, first, lens, offs)
    t_max = bench.reduce_max(float(rank + 1), world)
    t_sum = bench.reduce_sum(float(lens.sum()), world)
    dist.barrier()
    q.put((rank, first, len(lens), ct_d, tags, t_max, t_sum))
    dist.destroy_process_group()


@pytest.mark.parametrize("config", ["config2", "config3", "config4"])
def test_two_rank_shards_match_single_process(config):
    world, n = 2, 24
    if bench.CONFIGS[config][4] == "strong":
        n = 48  # the fixed batch, split in two
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, config, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    strong = bench.CONFIGS[config][4] == "strong"
    total = n if strong else world * n
    # shards are disjoint and contiguous and cover the batch
    assert res[0][1] == 0 and res[1][1] == res[0][2] and res[0][2] + res[1][2] == total
    # concatenation of per-rank results == one process sealing both shards
    sh = bench.shard_plan(config, 0, 1, records=total)
    all_ct, all_tags = _seal_shard(config, sh.first, sh.lens, sh.offs)
    assert res[0][4] + res[1][4] == all_tags
    n0 = res[0][2]
    sh0 = bench.shard_plan(config, 0, world, records=n)
    assert res[0][3] == _seal_shard(config, 0, sh.lens[:n0], sh0.offs)[0]
    # reductions
    assert all(r[5] == 2.0 for r in res)
    assert all(r[6] == float(sh.lens.sum()) for r in res)


def _plan(config, gpus, records=0):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"), "--gpus",
           str(gpus), "--plan-only", "--config", config]
    if records:
        cmd += ["--records", str(records)]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, out.stdout
    return json.loads(line[0])


@pytest.mark.parametrize("gpus", [2, 4, 8])
def test_launcher_config4_byte_balanced(gpus):
    """bench.py --gpus N starts N ranks itself; config 4 = ONE batch of 4M
    mixed-length records split into contiguous, byte-balanced ranges."""
    r = _plan("config4", gpus)
    assert r["n_gpus"] == gpus and r["scaling"] == "strong"
    plan = sorted(r["plan"], key=lambda x: x["rank"])
    assert [p["rank"] for p in plan] == list(range(gpus))
    pos = 0
    for p in plan:
        assert p["first"] == pos
        pos += p["n"]
    assert pos == 1 << 22
    all_bytes = int(bench.mixed_lengths(0, 1 << 22).sum())
    assert sum(p["bytes"] for p in plan) == all_bytes == r["reduce_sum"]
    mean = all_bytes / gpus
    # within about one record (the split is on 16-byte-padded lengths)
    assert max(abs(p["bytes"] - mean) for p in plan) <= 65536
    assert r["reduce_max"] == float(gpus)


@pytest.mark.parametrize("gpus", [2, 8])
def test_launcher_config5_key_ranges(gpus):
    """config 5 = ONE set of 64K keys x 64 records split by key ranges."""
    r = _plan("config5", gpus)
    plan = sorted(r["plan"], key=lambda x: x["rank"])
    assert sum(p["nkeys"] for p in plan) == 65536
    kpos = 0
    for p in plan:
        assert p["key_first"] == kpos and p["first"] == 64 * kpos and p["n"] == 64 * p["nkeys"]
        kpos += p["nkeys"]
    assert len({p["nkeys"] for p in plan}) == 1


def test_launcher_weak_config_per_gpu_shards():
    r = _plan("config2", 2, records=1000)
    plan = sorted(r["plan"], key=lambda x: x["rank"])
    assert r["scaling"] == "weak"
    assert [(p["first"], p["n"]) for p in plan] == [(0, 1000), (1000, 1000)]


def _parity_worker(rank, world, port, codes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    code = codes[rank]
    text = {bench.PARITY_OK: f"ref_digest_ok:shard{rank}",
            bench.PARITY_UNCHECKED: "not_checked:none",
            bench.PARITY_MISMATCH: f"MISMATCH:shard{rank}"}[code]
    q.put((rank,) + bench.reduce_parity(code, text, world, rank))
    dist.destroy_process_group()


@pytest.mark.parametrize("codes,expect", [
    ((2, 2, 2), "ref_digest_ok:all_ranks(3)"),
    ((2, 1, 2), "not_checked:1_of_3_ranks"),
    ((2, 1, 0), "MISMATCH:rank 2: MISMATCH:shard2")])
def test_parity_reduced_over_ranks(codes, expect):
    """bench.py's per-rank digest results are reduced over all ranks: the line
    says all_ranks only when every rank's shard matched its reference digest,
    and any mismatch (on any rank) is reported and fails the run."""
    world = len(codes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parity_worker, args=(r, world, port, codes, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, worst, summary, per_rank in res:
        assert worst == min(codes) and summary == expect
        assert len(per_rank) == world and per_rank[rank].startswith(f"rank {rank}:")
