#!/usr/bin/env python3
"""bench.py -- device-resident AEAD seal throughput on MI355X.

Metric (BASELINE.json): "GiB/s device-resident AEAD seal (AES-128-GCM, 16 KiB
records) at 1/2/4/8 GPUs".  Default workload = BASELINE config 2: AES-128-GCM
seal of 1,048,576 x 16 KiB synthetic records (16 GiB in, 16 GiB out, one key)
per GPU.  One step = one seal pass over the whole per-GPU batch, inputs
already resident in HBM.  Multi-GPU: one process per GPU; every rank seals
its own 1M-record shard (weak scaling, no collective on the data path); the
only collectives are the timing barrier and the max-over-ranks reduction.

Prints ONE JSON line on rank 0 (contract in the task description), including
`roofline` (algorithmic HBM bytes per launch / HIP-event kernel time vs the
8 TB/s HBM peak) and `cpu_baseline` (the reference library's CPU path,
oracle/_ref/ref_tool, on this host's cores, rank 0 at N=1 only).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import boringssl_amd as ba  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "GiB/s device-resident AEAD seal (AES-128-GCM, 16 KiB records) at 1/2/4/8 GPUs"

CONFIGS = {
    # name: (aead, key_len, records per GPU, record length or "mixed", description)
    # Only config2 is the BASELINE metric; the others are reported under their
    # own metric names.
    "config2": ("aes-128-gcm", 16, 1 << 20, 16384,
                "config2: AES-128-GCM seal, 1M x 16 KiB records per GPU, single key"),
    "config3": ("chacha20-poly1305", 32, 1 << 20, 1350,
                "config3: ChaCha20-Poly1305 seal, 1M x 1350 B records per GPU"),
    # XChaCha20-Poly1305: config 3's records with 24-byte
    # nonces (oracle/ref/ref_tool.cc make_nonce).
    "config3x": ("xchacha20-poly1305", 32, 1 << 20, 1350,
                 "config3x: XChaCha20-Poly1305 seal, 1M x 1350 B records per GPU"),
    # AES-GCM-SIV: config 2's records.
    "configS": ("aes-128-gcm-siv", 16, 1 << 20, 16384,
                "configS: AES-128-GCM-SIV seal, 1M x 16 KiB records per GPU, single key"),
    "config4": ("aes-256-gcm", 32, 1 << 22, "mixed",
                "config4: AES-256-GCM seal, 4M records of 64 B-16 KiB (mixed) per GPU"),
    # 64K keys x 64 records over 8 GPUs: per GPU 8192 keys x 64 records of
    # 16 KiB (BSSL_AMD_KEYSET, key_index per record, records grouped by key).
    "config5": ("aes-128-gcm", 16, 8192 * 64, 16384,
                "config5: AES-128-GCM seal, 8192 keys x 64 records x 16 KiB per GPU "
                "(64K keys over 8 GPUs), keyset"),
}
RECORDS_PER_KEY = {"config5": 64}


def synth_key(k, key_len):
    """oracle/synth.h key definition (host side, bench support only)."""
    out = bytearray()
    for b in range(key_len):
        x = (0xB055 + 16 * k + b // 8) & (2**64 - 1)
        z = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        z ^= z >> 31
        out.append((z >> (8 * (b % 8))) & 0xff)
    return bytes(out)


def mixed_lengths(first, n):
    i = np.arange(first, first + n, dtype=np.uint64)
    z = i + np.uint64(42) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return np.uint64(64) + z % np.uint64(16321)


METRICS = {
    "config2": METRIC,
    "config3": "GiB/s device-resident AEAD seal (ChaCha20-Poly1305, 1350 B records)",
    "config3x": "GiB/s device-resident AEAD seal (XChaCha20-Poly1305, 1350 B records)",
    "configS": "GiB/s device-resident AEAD seal (AES-128-GCM-SIV, 16 KiB records)",
    "config4": "GiB/s device-resident AEAD seal (AES-256-GCM, mixed 64 B-16 KiB records)",
    "config5": "GiB/s device-resident AEAD seal (AES-128-GCM, 16 KiB records, 64 records per key)",
}


def shard_plan(config, rank, world, records=0):
    """Records of rank `rank`: a disjoint shard [first, first + n) of the
    global record sequence (weak scaling: n records per GPU).  Returns
    (first, lengths[n], offsets[n], padded_total_bytes)."""
    aead, key_len, nrec, length, _ = CONFIGS[config]
    if records:
        nrec = records
    first = rank * nrec
    lens = mixed_lengths(first, nrec) if length == "mixed" else np.full(nrec, length, np.uint64)
    padded = (lens + np.uint64(15)) // np.uint64(16) * np.uint64(16)
    offs = np.zeros(nrec, dtype=np.uint64)
    offs[1:] = np.cumsum(padded[:-1])
    return first, lens, offs, int(padded.sum())


def reduce_max(value, world):
    """Max over ranks of a host float (the step time), via the process group."""
    if world == 1:
        return value
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
        else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(value, world):
    if world == 1:
        return value
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
        else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(aead, length, seconds):
    """Reference CPU path (oracle/_ref/ref_tool: the reference library built
    from /root/reference sources) on a bounded resident sample."""
    tool = os.path.join(ROOT, "oracle", "_ref", "ref_tool")
    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16")), 16)
    if isinstance(length, str):
        length = 8192
    nrec = max(1024, (1 << 30) // length)  # ~1 GiB resident sample
    if os.path.exists(tool):
        try:
            out = subprocess.check_output(
                [tool, "bench", aead, str(length), str(nrec), str(threads), str(seconds)],
                text=True, timeout=seconds * 4 + 120)
            r = json.loads(out)
            return {"value": round(r["gib_per_s"], 3), "unit": "GiB/s", "cores": threads,
                    "kind": "reference",
                    "sample": f"{nrec} synthetic records x {length} B (~1 GiB resident), "
                              f"{r['records_sealed']} seals in {r['seconds']:.1f} s, "
                              f"{threads} threads, reference EVP_AEAD_CTX_seal_scatter "
                              "(bench/aead.cc method, asm dispatch on this host)"}
        except Exception as e:  # pragma: no cover
            print(f"cpu baseline (reference) failed: {e}", file=sys.stderr)
    # Fallback: the C oracle restatement (a port, not the reference).
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as o
    n = 256
    pt, offs, nonces, ads = o.synth_batch(0, np.full(n, length, dtype=np.uint64))
    keys = np.frombuffer(synth_key(0, 16 if "128" in aead else 32), dtype=np.uint8).copy()
    out = np.zeros_like(pt)
    tags = np.zeros(16 * n, dtype=np.uint8)
    adoff = np.arange(n, dtype=np.uint64) * np.uint64(13)
    adl = np.full(n, 13, dtype=np.uint64)
    lens = np.full(n, length, dtype=np.uint64)
    aid = o.AES_GCM if "gcm" in aead else o.CHACHA20_POLY1305
    t0, done = time.time(), 0
    while time.time() - t0 < seconds:
        o.batch(aid, 1, keys, len(keys), None, pt, out, offs, lens, nonces, 12, ads, adoff, adl,
                tags, 16, None, threads)
        done += n
    dt = time.time() - t0
    return {"value": round(done * length / dt / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port", "sample": f"{done} records x {length} B via the C oracle"}


def load_traffic(kernel_prefix):
    """HBM bytes per launch from the rocprofv3 PMC pass (tools/pmc_traffic.py)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        for k, v in d.items():
            if k.startswith(kernel_prefix):
                return v.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="config2", choices=sorted(CONFIGS))
    ap.add_argument("--records", type=int, default=0, help="override records per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--op", default="seal", choices=["seal", "open"],
                    help="open: time EVP_AEAD open of the sealed batch (ct -> separate out)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    torch.cuda.set_device(local)
    ba.set_device(local)
    dev = torch.device(f"cuda:{local}")

    aead, key_len, _, length, desc = CONFIGS[args.config]
    first, lens, offs, total_pad = shard_plan(args.config, rank, world, args.records)
    nrec = len(lens)
    padded = (lens + np.uint64(15)) // np.uint64(16) * np.uint64(16)
    pt_bytes = int(lens.sum())

    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int64)).to(dev)
    d_pt = torch.empty(total_pad, dtype=torch.uint8, device=dev)
    d_ct = torch.empty(total_pad, dtype=torch.uint8, device=dev)
    d_nonce = torch.empty(12 * nrec, dtype=torch.uint8, device=dev)
    d_ad = torch.empty(13 * nrec, dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * nrec, dtype=torch.uint8, device=dev)
    d_status = torch.zeros(nrec, dtype=torch.uint8, device=dev)
    ba.synth_fill_device(first, nrec, d_offs, d_lens, d_pt, d_nonce, d_ad)
    nonce_len = 12
    if aead == "xchacha20-poly1305":  # 24-byte nonces (ref_tool.cc make_nonce)
        a = d_nonce.view(-1, 12)
        b = a.clone()
        b[:, 4:] ^= 0xff
        d_nonce, nonce_len = torch.cat([a, b], dim=1).contiguous().view(-1), 24
    uniform = length != "mixed"
    rpk = RECORDS_PER_KEY.get(args.config)
    d_kidx = None
    if rpk:
        # Keys of this rank's shard: global key ids first/rpk .. (synth_key).
        nkeys = (nrec + rpk - 1) // rpk
        k0 = first // rpk
        ctx = ba.Keyset(aead, b"".join(synth_key(k0 + k, key_len) for k in range(nkeys)), nkeys,
                        16)
        d_kidx = torch.from_numpy((np.arange(nrec) // rpk).astype(np.int32)).to(dev)
    else:
        ctx = ba.AEADCtx(aead, synth_key(0, key_len), 16)
    batch = ba.make_batch(nrec, d_pt, d_ct, d_tags, d_nonce, nonce_len, d_ad,
                          offsets=None if uniform else d_offs,
                          lengths=None if uniform else d_lens,
                          record_stride=int(padded[0]) if uniform else 0,
                          record_len=int(length) if uniform else 0,
                          ad_stride=13, ad_len=13, status=d_status, key_index=d_kidx)
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    op = ctx.seal_batch_device
    if args.op == "open":
        # Seal once, then time opens of the sealed records into a third buffer
        # (tags verified every step).
        ctx.seal_batch_device(batch, stream)
        d_back = torch.empty_like(d_pt)
        batch = ba.make_batch(nrec, d_ct, d_back, d_tags, d_nonce, nonce_len, d_ad,
                              offsets=None if uniform else d_offs,
                              lengths=None if uniform else d_lens,
                              record_stride=int(padded[0]) if uniform else 0,
                              record_len=int(length) if uniform else 0,
                              ad_stride=13, ad_len=13, status=d_status, key_index=d_kidx)
        op = ctx.open_batch_device

    for _ in range(args.warmup):
        op(batch, stream)
    torch.cuda.synchronize()
    if args.warmup and not bool(d_status.all()):
        raise SystemExit(f"{args.op} reported failed records")

    # Kernel-level timing: the library records HIP events on `stream`
    # immediately around the bulk kernel of every launch (no host sync).
    ba.set_kernel_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        op(batch, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = ba.collect_kernel_times()
    ba.set_kernel_timing(False)
    if not bool(d_status.all()):
        raise SystemExit(f"{args.op} reported failed records")
    if args.op == "open" and not torch.equal(d_back[:16 << 10], d_pt[:16 << 10]):
        raise SystemExit("open did not return the plaintext")
    assert len(kernel_ms) == args.steps, kernel_ms
    avg_kernel_ms = float(np.mean(kernel_ms))
    kname = ba.last_kernel_name()
    elapsed = reduce_max(elapsed, world)

    ms_per_step = elapsed * 1000.0 / args.steps
    total_bytes = reduce_sum(float(pt_bytes), world)  # all ranks' records
    value = total_bytes * args.steps / elapsed / 2**30
    algo_bytes = 2 * pt_bytes + (29 + nonce_len) * nrec  # PT in + CT out + tag + nonce + AD
    achieved = algo_bytes / (avg_kernel_ms / 1000.0) / 1e9
    traffic = load_traffic(kname)

    result = {
        "metric": METRICS[args.config] if args.op == "seal" else
                  METRICS[args.config].replace(" seal ", " open "),
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated records, oracle/synth.h definition)",
        "config": {"workload": desc, "aead": aead, "records_per_gpu": nrec,
                   "record_bytes": length, "plaintext_bytes_per_gpu": pt_bytes,
                   "parallelism": f"dp{world} (independent record shards, no collective)"},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "algorithmic_bytes_per_launch": algo_bytes,
                     "avg_kernel_ms": round(avg_kernel_ms, 4)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(aead, length, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
