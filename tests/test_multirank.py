"""Multi-rank (N>1) path on CPU with the gloo backend, world_size 2.

bench.py shards the record sequence across ranks (weak scaling, no data-path
collective): rank r seals records [r*n, (r+1)*n) with its own synthetic
inputs, and the only collectives are the timing barrier and max/sum
reductions.  This test runs those pieces on two gloo ranks and checks that the
per-rank seals (done here by the CPU oracle, the checker) concatenate to
exactly the single-process result, and that the reductions are max/sum.
"""
import hashlib
import os
import socket

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
    pt, offs2, nonces, ads = o.synth_batch(first, lens)
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
    first, lens, offs, _ = bench.shard_plan(config, rank, world, records=n)
    ct_d, tags = _seal_shard(config, first, lens, offs)
    t_max = bench.reduce_max(float(rank + 1), world)
    t_sum = bench.reduce_sum(float(lens.sum()), world)
    dist.barrier()
    q.put((rank, first, len(lens), ct_d, tags, t_max, t_sum))
    dist.destroy_process_group()


@pytest.mark.parametrize("config", ["config2", "config3", "config4"])
def test_two_rank_shards_match_single_process(config):
    world, n = 2, 24
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
    # shards are disjoint and contiguous
    assert [r[1] for r in res] == [0, n] and all(r[2] == n for r in res)
    # concatenation of per-rank results == one process sealing both shards
    first, lens, offs, _ = bench.shard_plan(config, 0, 1, records=world * n)
    all_ct, all_tags = _seal_shard(config, first, lens, offs)
    assert res[0][4] + res[1][4] == all_tags
    lens0 = lens[:n]
    # ciphertext digests per shard
    pt, offs_all, nonces, ads = o.synth_batch(0, lens)
    assert res[0][3] == _seal_shard(config, 0, lens0, offs[:n])[0]
    # reductions
    assert all(r[5] == 2.0 for r in res)
    assert all(r[6] == float(lens.sum()) for r in res)
