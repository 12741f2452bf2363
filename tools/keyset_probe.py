#!/usr/bin/env python3
"""Where config 5 (64K keys x 64 records of 16 KiB, the keyset kernel) loses
against config 2: the same batch timed (a) as the bench runs it, (b) with
every record on key 0 (the same tiles and passes, but no GHASH table rebuild
and no key change between tiles), (c) through the one-key kernel (a context
of key 0: dynamic units, no tiles).  Prints one JSON line of GiB/s.  (b) and
(c) seal with other keys than the bench's, so only (a) is digest-checked.

Usage: python tools/keyset_probe.py [--records 4194304] [--steps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import boringssl_amd as ba  # noqa: E402


def timed(fn, steps):
    s = torch.cuda.current_stream()
    fn(s)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(steps):
        fn(s)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=64 * 65536)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    w = bench.build_workload("config5", 0, 1, args.records, dev)
    gib = w.pt_bytes / 2**30
    out = {}
    out["a_keyset"] = gib / timed(lambda s: w.op(w.batch, s), args.steps) * 1e3
    code, parity = bench.verify_workload(w)
    out["a_parity"] = parity
    # (b) key_index all zeros: the batch's key_index tensor is the last ref.
    kidx = w.batch._refs[-1]
    saved = kidx.clone()
    kidx.zero_()
    out["b_keyset_one_key"] = gib / timed(lambda s: w.op(w.batch, s), args.steps) * 1e3
    kidx.copy_(saved)
    # (c) the same records through the one-key kernel.
    ctx = ba.AEADCtx("aes-128-gcm", bench.synth_key(0, 16), 16)
    b = w.batch
    b.key_index = None
    out["c_one_key_kernel"] = gib / timed(lambda s: ctx.seal_batch_device(b, s), args.steps) * 1e3
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out.items()}))


if __name__ == "__main__":
    main()
