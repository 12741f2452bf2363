#!/usr/bin/env python3
"""bench.py -- device-resident AEAD seal throughput on MI355X.

Metric (BASELINE.json): "GiB/s device-resident AEAD seal (AES-128-GCM, 16 KiB
records) at 1/2/4/8 GPUs".  Default workload = BASELINE config 2: AES-128-GCM
seal of 1,048,576 x 16 KiB synthetic records (16 GiB in, 16 GiB out, one key)
per GPU.  One step = one seal pass over the whole per-GPU batch, inputs
already resident in HBM.

Multi-GPU: one process per GPU, records sharded with no
collective on the data path; the only collectives are the timing barrier, the
max of the step time and the sum of the bytes.
  * `python bench.py --gpus N` (WORLD_SIZE unset) starts N rank processes
    itself, before anything touches a GPU, and prints rank 0's line;
    under `torch.distributed.run` each rank reads RANK/LOCAL_RANK/WORLD_SIZE.
  * configs 2, 3, 3x, S are per-GPU workloads (weak scaling: 1M records per
    GPU); config 4 is ONE fixed batch of 4M mixed-length records split into
    contiguous ranges balanced by bytes (prefix sum of the record lengths), and
    config 5 is ONE fixed set of 64K keys x 64 records split by key ranges
    (strong scaling: the total work is fixed as N grows).
  * `--plan-only` runs the launcher, the rendezvous, the shard plan and the
    reductions on CPU (gloo) without a GPU (tests/test_multirank.py).

Prints ONE JSON line on rank 0 (contract in the task description), including
`roofline` (algorithmic HBM bytes per launch / HIP-event kernel time vs the
8 TB/s HBM peak) and `cpu_baseline` (the reference library's CPU path,
oracle/_ref/ref_tool bench1 = bench/aead.cc's BM_SpeedAEAD, one pinned
process per physical host core, rank 0 at N=1 only).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "GiB/s device-resident AEAD seal (AES-128-GCM, 16 KiB records) at 1/2/4/8 GPUs"

CONFIGS = {
    # name: (aead, key_len, records, record length or "mixed", scaling, description)
    # Weak configs: `records` per GPU.  Strong configs: `records` in total,
    # split across the GPUs.  Only config2 is the BASELINE metric; the others
    # are reported under their own metric names.
    "config2": ("aes-128-gcm", 16, 1 << 20, 16384, "weak",
                "config2: AES-128-GCM seal, 1M x 16 KiB records per GPU, single key"),
    "config3": ("chacha20-poly1305", 32, 1 << 20, 1350, "weak",
                "config3: ChaCha20-Poly1305 seal, 1M x 1350 B records per GPU"),
    # XChaCha20-Poly1305: config 3's records with 24-byte
    # nonces (oracle/ref/ref_tool.cc make_nonce).
    "config3x": ("xchacha20-poly1305", 32, 1 << 20, 1350, "weak",
                 "config3x: XChaCha20-Poly1305 seal, 1M x 1350 B records per GPU"),
    # AES-128-GCM on config 3's TLS-MTU records (per-record cost of the GCM
    # kernel: the record start and the tag, not in config 2's 16 KiB records).
    "configG": ("aes-128-gcm", 16, 1 << 20, 1350, "weak",
                "configG: AES-128-GCM seal, 1M x 1350 B records per GPU"),
    # AES-GCM-SIV: config 2's records.
    "configS": ("aes-128-gcm-siv", 16, 1 << 20, 16384, "weak",
                "configS: AES-128-GCM-SIV seal, 1M x 16 KiB records per GPU, single key"),
    "config4": ("aes-256-gcm", 32, 1 << 22, "mixed", "strong",
                "config4: AES-256-GCM seal, one batch of 4M records of 64 B-16 KiB (mixed), "
                "split across the GPUs by bytes"),
    # 64K keys x 64 records of 16 KiB (BSSL_AMD_KEYSET, key_index per record,
    # records grouped by key), split across the GPUs by key ranges.
    "config5": ("aes-128-gcm", 16, 65536 * 64, 16384, "strong",
                "config5: AES-128-GCM seal, 64K keys x 64 records x 16 KiB (keyset), "
                "split across the GPUs by key ranges"),
}
RECORDS_PER_KEY = {"config5": 64}

METRICS = {
    "config2": METRIC,
    "config3": "GiB/s device-resident AEAD seal (ChaCha20-Poly1305, 1350 B records)",
    "config3x": "GiB/s device-resident AEAD seal (XChaCha20-Poly1305, 1350 B records)",
    "configS": "GiB/s device-resident AEAD seal (AES-128-GCM-SIV, 16 KiB records)",
    "configG": "GiB/s device-resident AEAD seal (AES-128-GCM, 1350 B records)",
    "config4": "GiB/s device-resident AEAD seal (AES-256-GCM, mixed 64 B-16 KiB records)",
    "config5": "GiB/s device-resident AEAD seal (AES-128-GCM, 16 KiB records, 64 records per key)",
}


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
    """oracle/synth.h synth_mixed_len for records first .. first+n-1."""
    i = np.arange(first, first + n, dtype=np.uint64)
    z = i + np.uint64(42) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return np.uint64(64) + z % np.uint64(16321)


def _pad16(lens, align=16):
    a = np.uint64(align)
    return (lens + a - np.uint64(1)) // a * a


# Record alignment of the batch layout (bytes; BSSL_AMD_ALIGN overrides): no
# two records share a 128-byte cache line.  Config 3 (1350-byte records, so a
# 1408- instead of 1360-byte stride) measured 1,130-1,136 GiB/s against
# 1,091-1,124 for 16-byte alignment on one box, counted traffic within 2 %
# (DESIGN.md 4.3); 16 KiB records are unaffected.  Algorithmic bytes do not
# count the padding.
def record_align(config):
    return int(os.environ.get("BSSL_AMD_ALIGN", 128))


class Shard:
    """Records [first, first + n) of the global record sequence on one rank.
    `lens`/`offs` describe the rank's packed batch (records aligned to
    `align` bytes, record_align)."""

    def __init__(self, first, lens, key_first=0, nkeys=0, align=16):
        self.first = int(first)
        self.lens = lens
        padded = _pad16(lens, align)
        self.offs = np.zeros(len(lens), dtype=np.uint64)
        if len(lens):
            self.offs[1:] = np.cumsum(padded[:-1])
        self.total_pad = int(padded.sum())
        self.key_first, self.nkeys = key_first, nkeys

    @property
    def n(self):
        return len(self.lens)


def byte_balanced_split(lens, world):
    """Split points s_0 = 0 <= s_1 <= ... <= s_world = n of a record sequence
    into contiguous ranges of nearly equal bytes: s_r is the first record whose
    exclusive prefix sum of (padded) lengths reaches r/world of the total."""
    prefix = np.zeros(len(lens) + 1, dtype=np.float64)
    prefix[1:] = np.cumsum(_pad16(lens).astype(np.float64))
    targets = prefix[-1] * np.arange(world + 1) / world
    s = np.searchsorted(prefix, targets, side="left")
    s[0], s[-1] = 0, len(lens)
    return [int(x) for x in s]


def shard_plan(config, rank, world, records=0):
    """The records of rank `rank` of `world`.

    Weak configs: rank r seals records [r*n, (r+1)*n) of the synthetic
    sequence (n = `records` or the config's per-GPU count).  config4: the fixed
    batch of `records` (default 4M) mixed-length records, split by bytes.
    config5: the fixed 64K keys (or records/64) split by key ranges."""
    aead, key_len, nrec, length, scaling, _ = CONFIGS[config]
    if records:
        nrec = records
    if scaling == "weak":
        first = rank * nrec
        lens = mixed_lengths(first, nrec) if length == "mixed" else np.full(nrec, length,
                                                                            np.uint64)
        return Shard(first, lens, align=record_align(config))
    if config in RECORDS_PER_KEY:
        rpk = RECORDS_PER_KEY[config]
        nkeys_total = nrec // rpk
        k0, k1 = nkeys_total * rank // world, nkeys_total * (rank + 1) // world
        return Shard(k0 * rpk, np.full((k1 - k0) * rpk, length, np.uint64), k0, k1 - k0,
                     align=record_align(config))
    all_lens = mixed_lengths(0, nrec) if length == "mixed" else np.full(nrec, length, np.uint64)
    s = byte_balanced_split(all_lens, world)
    return Shard(s[rank], all_lens[s[rank]:s[rank + 1]].copy(), align=record_align(config))


# ---------------------------------------------------------------------------
# rank-process launcher (python bench.py --gpus N without torch.distributed.run)

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, timeout=None):
    """Start n rank processes of this script (one per GPU) and wait for them.
    Runs before anything in this process touches a GPU; the children are
    fresh processes (never exec).  Rank 0's stdout is passed through; the other
    ranks' stdout goes to temporary files whose last line is echoed to stderr
    when the rank ends.  If a rank fails, or the whole launch exceeds `timeout`
    seconds (BSSL_AMD_RANK_TIMEOUT, default 1800), every remaining rank is
    terminated (then killed) and the exit code is non-zero (124 on timeout).
    Returns the exit code."""
    import tempfile
    if timeout is None:
        timeout = float(os.environ.get("BSSL_AMD_RANK_TIMEOUT", "1800"))
    port = _free_port()
    procs, logs = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        log = None if r == 0 else tempfile.TemporaryFile(mode="w+")
        logs.append(log)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=log))

    def stop_all(live):
        for q in live:
            q.terminate()
        t_end = time.time() + 10
        for q in live:
            try:
                q.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                q.kill()

    rc = 0
    live = list(procs)
    deadline = time.time() + timeout
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                stop_all(live)
                live = []
                break
        if live and time.time() > deadline:
            print(f"bench.py: ranks still running after {timeout:.0f} s; stopping them",
                  file=sys.stderr)
            rc = 124
            stop_all(live)
            live = []
        time.sleep(0.05)
    for r, (p, log) in enumerate(zip(procs, logs)):
        p.wait()
        if log is not None:
            log.seek(0)
            lines = [x for x in log.read().splitlines() if x.strip()]
            log.close()
            print(f"bench.py: rank {r} exit {p.returncode}; last line: "
                  f"{lines[-1] if lines else '(none)'}", file=sys.stderr)
        if p.returncode not in (0, None) and rc == 0:
            rc = p.returncode
    return rc if rc >= 0 else 128 - rc


# ---------------------------------------------------------------------------
# reductions over ranks (timing only; no data-path collective)

def _dist():
    import torch.distributed as dist
    return dist


def _reduce(value, world, op):
    if world == 1:
        return value
    import torch
    dist = _dist()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
        else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def reduce_max(value, world):
    """Max over ranks of a host float (the step time), via the process group."""
    return _reduce(value, world, _dist().ReduceOp.MAX if world > 1 else None)


def reduce_sum(value, world):
    return _reduce(value, world, _dist().ReduceOp.SUM if world > 1 else None)


# ---------------------------------------------------------------------------
# CPU baseline

def physical_cores(limit=16):
    """One logical CPU per physical core of this process's affinity set,
    at most `limit` (the box's CPU share for one GPU)."""
    seen, cores = set(), []
    for c in sorted(os.sched_getaffinity(0)):
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                sib = f.read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            cores.append(c)
    return cores[:limit]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _pinned_runs(cmd, cores, timeout):
    procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True,
                              preexec_fn=(lambda c=c: os.sched_setaffinity(0, {c})))
             for c in cores]
    out = []
    for p in procs:
        o, _ = p.communicate(timeout=timeout)
        if p.returncode != 0:
            raise RuntimeError(f"{cmd} exited {p.returncode}")
        out.append(json.loads(o))
    return out


def cpu_baseline(aead, length, seconds):
    """The reference CPU path timed on this host: oracle/_ref/ref_tool bench1
    (the reference library built from /root/reference sources, driven exactly
    as bench/aead.cc:41-133 BM_SpeedAEAD drives it: one EVP_AEAD_CTX, zero
    key/nonce/13-byte AD/input, the same 16-byte-aligned buffer resealed, so
    the data is cache-resident) as one single-threaded process pinned to each
    physical core, seal and open.  value = the sum over cores (whole host)."""
    tool = os.path.join(ROOT, "oracle", "_ref", "ref_tool")
    if isinstance(length, str):  # mixed 64 B-16 KiB: bench/aead.cc's 8192-byte size
        length = 8192
    cores = physical_cores()
    if os.path.exists(tool):
        try:
            res = {}
            for op in ("seal", "open"):
                runs = _pinned_runs([tool, "bench1", aead, op, str(length), str(seconds)], cores,
                                    seconds * 4 + 60)
                v = [r["gib_per_s"] for r in runs]
                res[op] = (sum(v), sum(v) / len(v), min(v), max(v))
            return {"value": round(res["seal"][0], 3), "unit": "GiB/s", "cores": len(cores),
                    "kind": "reference",
                    "per_core": round(res["seal"][1], 3),
                    "per_core_min_max": [round(res["seal"][2], 3), round(res["seal"][3], 3)],
                    "open": {"value": round(res["open"][0], 3),
                             "per_core": round(res["open"][1], 3)},
                    "cpu_model": cpu_model(),
                    "sample": f"BM_SpeedAEAD method (bench/aead.cc:41-133): {aead} seal and open "
                              f"of one {length}-byte input, 13-byte AD, resealed for {seconds} s, "
                              f"one single-threaded process pinned per physical core x "
                              f"{len(cores)} cores (cache-resident, as the reference bench; the "
                              f"GPU value is HBM-resident)"}
        except Exception as e:  # pragma: no cover
            print(f"cpu baseline (reference) failed: {e}", file=sys.stderr)
    # Fallback: the C oracle restatement (a port, not the reference), one thread.
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as o
    n = 64
    lens = np.full(n, length, dtype=np.uint64)
    pt, offs, nonces, ads = o.synth_batch(0, lens)
    keys = np.frombuffer(synth_key(0, 16 if "128" in aead else 32), dtype=np.uint8).copy()
    out = np.zeros_like(pt)
    tags = np.zeros(16 * n, dtype=np.uint8)
    adoff = np.arange(n, dtype=np.uint64) * np.uint64(13)
    adl = np.full(n, 13, dtype=np.uint64)
    aid = o.AES_GCM if "gcm" in aead else o.CHACHA20_POLY1305
    t0, done = time.time(), 0
    while time.time() - t0 < seconds:
        o.batch(aid, 1, keys, len(keys), None, pt, out, offs, lens, nonces, 12, ads, adoff, adl,
                tags, 16, None, 1)
        done += n
    dt = time.time() - t0
    return {"value": round(done * length / dt / 2**30, 4), "unit": "GiB/s", "cores": 1,
            "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{done} records x {length} B via the C oracle, one thread"}


def load_profile(config, kernel_prefix):
    """HBM bytes per launch and LDS/VALU busy fractions of `config`'s bulk
    kernel from the rocprofv3 PMC passes (tools/profile_r02.sh ->
    tools/pmc_traffic.py -> profiles/traffic.json)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p)).get(config, {})
        # (the keyset kernel of config 5 is a gcm_kernel for the bench line)
        # (the table-free engine's lines: gcm_bs_kernel, config 5 gcm_bs_keyset_kernel)
        family = ("gcm_kernel", "gcm_keyset_kernel") if kernel_prefix == "gcm_kernel" else \
            ("gcm_bs_kernel", "gcm_bs_keyset_kernel") if kernel_prefix == "gcm_bs_kernel" else \
            (kernel_prefix,)
        for k, v in d.items():
            if isinstance(v, dict) and k.startswith(family):
                cb = {x: round(v[x], 3) for x in ("lds_busy", "valu_busy") if x in v}
                if cb:
                    cb["source"] = f"profiles/traffic.json[{config}] (rocprofv3 PMC)"
                # HBM bytes: FETCH_SIZE / WRITE_SIZE scaled by the calibration
                # copy of the kernel's record access pattern when the profile
                # has one (tools/micro/calib_copy), else the guide's x2 rule.
                if v.get("hbm_bytes_calibrated"):
                    if cb:
                        cb["traffic_rule"] = f"calibrated ({v.get('calib_pattern', '?')})"
                    return v["hbm_bytes_calibrated"], cb or None
                if cb:
                    cb["traffic_rule"] = "FETCH_SIZE x2 (guide)"
                return v.get("hbm_bytes_per_launch"), cb or None
    except Exception:
        return None, None
    return None, None


# ---------------------------------------------------------------------------

class Workload:
    """Device buffers and the batch descriptor of one rank's bench batch."""


def build_workload(config, rank, world, records, dev, open_op=False):
    """The rank's batch exactly as the bench times it: synthetic records
    (oracle/synth.h) generated in HBM, uniform configs as a uniform layout
    (record_stride / record_len, no per-record arrays), records aligned to
    record_align() bytes; config 4 with per-record offsets/lengths; config 5 a
    keyset with key_index.  open_op: seal once, then time opens of the sealed
    batch into a third buffer.  Used by main() and by the parity tests
    (tests/test_bench_layout.py), so the timed layout is the tested one."""
    import torch
    import boringssl_amd as ba
    aead, key_len, _, length, scaling, _ = CONFIGS[config]
    sh = shard_plan(config, rank, world, records)
    first, lens, offs, nrec = sh.first, sh.lens, sh.offs, sh.n
    padded = _pad16(lens, record_align(config))
    w = Workload()
    w.config, w.aead, w.shard, w.nrec, w.lens, w.offs = config, aead, sh, nrec, lens, offs
    w.pt_bytes = int(lens.sum())
    w.world = world
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int64)).to(dev)
    # Base offset of the record buffers within their allocation (bytes;
    # BSSL_AMD_BASE_OFFSET, diagnostic): shifts every record's cache-line phase.
    boff = int(os.environ.get("BSSL_AMD_BASE_OFFSET", 0))
    # Zero-filled, so the padding between records is defined (the kernels never
    # write it; the open check compares whole buffers).
    w.d_pt = torch.zeros(max(1, sh.total_pad) + boff, dtype=torch.uint8, device=dev)[boff:]
    w.d_ct = torch.zeros(max(1, sh.total_pad) + boff, dtype=torch.uint8, device=dev)[boff:]
    d_nonce = torch.empty(max(1, 12 * nrec), dtype=torch.uint8, device=dev)
    d_ad = torch.empty(max(1, 13 * nrec), dtype=torch.uint8, device=dev)
    w.d_tags = torch.empty(max(1, 16 * nrec), dtype=torch.uint8, device=dev)
    w.d_status = torch.zeros(max(1, nrec), dtype=torch.uint8, device=dev)
    ba.synth_fill_device(first, nrec, d_offs, d_lens, w.d_pt, d_nonce, d_ad)
    nonce_len = 12
    if aead == "xchacha20-poly1305":  # 24-byte nonces (ref_tool.cc make_nonce)
        a = d_nonce.view(-1, 12)
        b = a.clone()
        b[:, 4:] ^= 0xff
        d_nonce, nonce_len = torch.cat([a, b], dim=1).contiguous().view(-1), 24
    w.nonce_len = nonce_len
    w.uniform = uniform = length != "mixed"
    rpk = RECORDS_PER_KEY.get(config)
    d_kidx = None
    w.nkeys = 1
    if rpk:
        # The rank's keys: global key ids key_first .. (synth_key).
        w.nkeys = sh.nkeys
        ctx = ba.Keyset(aead, b"".join(synth_key(sh.key_first + k, key_len)
                                       for k in range(sh.nkeys)), sh.nkeys, 16)
        d_kidx = torch.from_numpy((np.arange(nrec) // rpk).astype(np.int32)).to(dev)
    else:
        ctx = ba.AEADCtx(aead, synth_key(0, key_len), 16)
    w.ctx = ctx
    w.stride = stride = int(padded[0]) if nrec else 16

    def mk(src, dst):
        return ba.make_batch(nrec, src, dst, w.d_tags, d_nonce, nonce_len, d_ad,
                             offsets=None if uniform else d_offs,
                             lengths=None if uniform else d_lens,
                             record_stride=stride if uniform else 0,
                             record_len=int(length) if uniform else 0,
                             ad_stride=13, ad_len=13, status=w.d_status, key_index=d_kidx)
    w.batch = mk(w.d_pt, w.d_ct)
    w.op = ctx.seal_batch_device
    torch.cuda.synchronize()
    if open_op:
        ctx.seal_batch_device(w.batch, torch.cuda.current_stream())
        w.d_back = torch.zeros(w.d_pt.numel() + boff, dtype=torch.uint8, device=dev)[boff:]
        w.batch = mk(w.d_ct, w.d_back)
        w.op = ctx.open_batch_device
        torch.cuda.synchronize()
    return w


def shard_key(aead, length, first, n, rpk):
    """Identity of a reference digest of records [first, first + n) of the
    synthetic sequence (key i // rpk, rpk 0 = one key; tests/golden/
    make_golden.py shard_key, oracle/ref/ref_tool.cc cmd_shard)."""
    return f"{aead}/{length}/first={first}/n={n}/rpk={rpk}"


def golden_entry(w):
    """The reference digest of the rank's batch, or None.  Any shard of any
    rank: tests/golden/ref_shard_digests.json holds the reference library's
    digest of every rank's records at N = 2, 4, 8 (matched by first record,
    record count, records per key, length); tests/golden/ref_digests.json the
    whole N = 1 workloads (first record 0)."""
    length = CONFIGS[w.config][3]
    rpk = RECORDS_PER_KEY.get(w.config, 0)
    gdir = os.path.join(ROOT, "tests", "golden")
    try:
        with open(os.path.join(gdir, "ref_shard_digests.json")) as f:
            shards = json.load(f)
    except OSError:
        shards = {}
    key = shard_key(w.aead, length, w.shard.first, w.nrec, rpk)
    if key in shards:
        return key, shards[key]
    if w.shard.first != 0 or w.shard.key_first != 0:
        return None
    try:
        with open(os.path.join(gdir, "ref_digests.json")) as f:
            golden = json.load(f)
    except OSError:
        return None
    rpk_full = rpk or w.nrec
    for name, g in sorted(golden.items()):
        if (g["aead"] == w.aead and int(g["records"]) == w.nrec and int(g["nkeys"]) == w.nkeys
                and int(g["records_per_key"]) == rpk_full and str(g["len"]) == str(length)):
            return name, g
    return None


def device_digests(d_out, offs, lens, d_tags, uniform_stride=0, chunk=1024, threads=16):
    """(tags_sha256, ct_sha256) of sealed records on the device, with the
    reference tool's definition (oracle/ref/ref_tool.cc cmd_digest; as
    tests/golden_util.batch_digests): SHA-256 over all tags in record order,
    and SHA-256 over the per-1024-record SHA-256 of the concatenated
    ciphertexts.  Streams the records to the host chunk by chunk."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    n = len(lens)
    L = int(lens[0]) if n else 0

    def part(c):
        lo, hi = c * chunk, min(n, (c + 1) * chunk)
        lo_b, hi_b = int(offs[lo]), int(offs[hi - 1] + lens[hi - 1])
        host = d_out[lo_b:hi_b].cpu().numpy()
        if uniform_stride:
            if uniform_stride == L:
                data = host.tobytes()
            else:
                full = np.zeros((hi - lo) * uniform_stride, dtype=np.uint8)
                full[:host.size] = host
                data = full.reshape(hi - lo, uniform_stride)[:, :L].tobytes()
        else:
            data = b"".join(host[int(offs[i]) - lo_b:int(offs[i]) - lo_b + int(lens[i])].tobytes()
                            for i in range(lo, hi))
        return hashlib.sha256(data).digest()

    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(part, range((n + chunk - 1) // chunk)))
    tags = d_tags[:16 * n].cpu().numpy().tobytes()
    return hashlib.sha256(tags).hexdigest(), hashlib.sha256(b"".join(parts)).hexdigest()


PARITY_MISMATCH, PARITY_UNCHECKED, PARITY_OK = 0, 1, 2


def verify_workload(w):
    """Compare the rank's sealed batch with the reference library's digest of
    the same records.  Returns (code, text): (PARITY_OK, "ref_digest_ok:<entry>"),
    (PARITY_UNCHECKED, "not_checked:<reason>") or (PARITY_MISMATCH, "MISMATCH:...")
    -- the caller reduces the codes over ranks and fails the run on a mismatch."""
    ge = golden_entry(w)
    if ge is None:
        return PARITY_UNCHECKED, "not_checked:no reference digest for this shard"
    name, g = ge
    tags_d, ct_d = device_digests(w.d_ct, w.offs, w.lens, w.d_tags,
                                  uniform_stride=w.stride if w.uniform else 0)
    if tags_d != g["tags_sha256"] or ct_d != g["ct_sha256"]:
        return PARITY_MISMATCH, (f"MISMATCH:{name} (tags {tags_d[:16]} vs "
                                 f"{g['tags_sha256'][:16]}, ct {ct_d[:16]} vs {g['ct_sha256'][:16]})")
    return PARITY_OK, f"ref_digest_ok:{name}"


def reduce_parity(code, text, world, rank):
    """All ranks' parity results: (min code over ranks, summary string, per-rank
    list).  "ref_digest_ok:all_ranks" when every rank's shard matched the
    reference digest (per-GPU digests, combined on the host in
    rank order)."""
    if world == 1:
        return code, text, [text]
    texts = [None] * world
    _dist().all_gather_object(texts, f"rank {rank}: {text}")
    worst = int(round(_reduce(float(code), world, _dist().ReduceOp.MIN)))
    if worst == PARITY_OK:
        summary = f"ref_digest_ok:all_ranks({world})"
    elif worst == PARITY_UNCHECKED:
        n_un = sum(1 for t in texts if "not_checked" in t)
        summary = f"not_checked:{n_un}_of_{world}_ranks"
    else:
        summary = "MISMATCH:" + "; ".join(t for t in texts if "MISMATCH" in t)
    return worst, summary, texts


def plan_only(args, world, rank):
    """The launcher/plan/reduction path without a GPU (gloo)."""
    dist = _dist()
    if world > 1:
        dist.init_process_group("gloo")
    sh = shard_plan(args.config, rank, world, args.records)
    mine = {"rank": rank, "first": sh.first, "n": sh.n, "bytes": int(sh.lens.sum()),
            "key_first": sh.key_first, "nkeys": sh.nkeys}
    plans = [mine]
    if world > 1:
        plans = [None] * world
        dist.all_gather_object(plans, mine)
    t_max = reduce_max(float(rank + 1), world)
    total = reduce_sum(float(mine["bytes"]), world)
    if rank == 0:
        print(json.dumps({"plan_only": True, "config": args.config, "n_gpus": world,
                          "scaling": CONFIGS[args.config][4], "plan": plans,
                          "reduce_max": t_max, "reduce_sum": total}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="config2", choices=sorted(CONFIGS))
    ap.add_argument("--records", type=int, default=0,
                    help="override the record count (per GPU for weak configs, total for "
                         "config4/config5)")
    ap.add_argument("--cpu-seconds", type=float, default=5.0,
                    help="seconds per CPU-baseline measurement (seal, then open)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the digest check of the sealed output after the timed steps")
    ap.add_argument("--plan-only", action="store_true",
                    help="launcher + shard plan + reductions on CPU (gloo), no GPU")
    ap.add_argument("--op", default="seal", choices=["seal", "open"],
                    help="open: time EVP_AEAD open of the sealed batch (ct -> separate out)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}",
              file=sys.stderr)
    if args.plan_only:
        plan_only(args, world, rank)
        return

    import torch
    import boringssl_amd as ba  # fails loudly without the HIP library

    dist = _dist()
    # Rehearsal on fewer GPUs than ranks (diagnostic; BSSL_AMD_REHEARSE_DEVICES
    # = k): rank r uses GPU r mod k, and the timing collectives run over gloo
    # (RCCL does not put two ranks of one communicator on one GPU).
    rehearse = int(os.environ.get("BSSL_AMD_REHEARSE_DEVICES", "0"))
    if rehearse:
        local %= rehearse
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    torch.cuda.set_device(local)
    ba.set_device(local)
    dev = torch.device(f"cuda:{local}")

    aead, key_len, _, length, scaling, desc = CONFIGS[args.config]
    wl = build_workload(args.config, rank, world, args.records, dev, open_op=args.op == "open")
    sh, nrec, pt_bytes, nonce_len = wl.shard, wl.nrec, wl.pt_bytes, wl.nonce_len
    d_status, batch, op = wl.d_status, wl.batch, wl.op
    stream = torch.cuda.current_stream()

    for _ in range(args.warmup):
        op(batch, stream)
    torch.cuda.synchronize()
    if args.warmup and nrec and not bool(d_status[:nrec].all()):
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
    if nrec and not bool(d_status[:nrec].all()):
        raise SystemExit(f"{args.op} reported failed records")
    if args.op == "open" and not torch.equal(wl.d_back, wl.d_pt):
        raise SystemExit("open did not return the plaintext")
    # Bit-exact check of the timed output (seal), on every rank: the digest of
    # the rank's sealed records and tags against the reference library's
    # digest of the same records (tests/golden/ref_shard_digests.json,
    # ref_digests.json); reduced over ranks below.
    if args.op == "seal" and not args.no_parity:
        p_code, p_text = verify_workload(wl)
    else:
        p_code, p_text = PARITY_UNCHECKED, "not_checked"
    p_code, parity, parity_ranks = reduce_parity(p_code, p_text, world, rank)
    assert len(kernel_ms) == args.steps, kernel_ms
    avg_kernel_ms = float(np.mean(kernel_ms))
    kname = ba.last_kernel_name()
    elapsed = reduce_max(elapsed, world)

    ms_per_step = elapsed * 1000.0 / args.steps
    total_bytes = reduce_sum(float(pt_bytes), world)  # all ranks' records
    value = total_bytes * args.steps / elapsed / 2**30
    algo_bytes = 2 * pt_bytes + (29 + nonce_len) * nrec  # PT in + CT out + tag + nonce + AD
    achieved = algo_bytes / (avg_kernel_ms / 1000.0) / 1e9
    traffic, compute_bound = load_profile(args.config, kname)
    if world > 1 or args.records or args.op != "seal":
        traffic, compute_bound = None, None  # the profile is of the default N=1 seal run

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
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated records, oracle/synth.h definition)",
        "config": {"workload": desc, "aead": aead,
                   "records_per_gpu" if scaling == "weak" else "records_rank0": nrec,
                   "record_bytes": length, "plaintext_bytes_rank0": pt_bytes,
                   "plaintext_bytes_all_ranks": int(total_bytes),
                   "parallelism": f"dp{world} (independent record shards, no collective)"},
        "parity": parity,
        **({"parity_ranks": parity_ranks} if world > 1 else {}),
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "algorithmic_bytes_per_launch": algo_bytes,
                     "avg_kernel_ms": round(avg_kernel_ms, 4),
                     "compute_bound": compute_bound},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(aead, length, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if p_code == PARITY_MISMATCH:
        raise SystemExit(f"bench.py: sealed output differs from the reference digest: {parity}")


if __name__ == "__main__":
    main()
