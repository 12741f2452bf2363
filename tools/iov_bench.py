#!/usr/bin/env python3
"""Throughput of EVP_AEAD_CTX_sealv_batch_device (device iovec records,
iovec.hip) next to the contiguous batch on the same records (aligned; at the iovec
layout's odd stride in place and into a second arena), and the iovec batch in
place.

Each record is split into three chunks as a socket layer would hand it over
(a 5-byte piece, the middle, the rest), the chunks packed back to back at odd
offsets in one arena (so most chunks are unaligned), outputs to a second
arena; AD is one 13-byte chunk per record.  Prints one JSON line.

  python tools/iov_bench.py [--aead aes-128-gcm] [--records N] [--len L] [--steps K]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import boringssl_amd as ba  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--aead", default="aes-128-gcm")
    ap.add_argument("--records", type=int, default=1 << 18)
    ap.add_argument("--len", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--in-gap", type=int, default=1,
                    help="bytes between input records (1: record starts at every alignment)")
    ap.add_argument("--out-gap", type=int, default=1, help="the same for the outputs")
    ap.add_argument("--cut1", type=int, default=5, help="length of each record's first chunk")
    ap.add_argument("--cut2", type=int, default=-1,
                    help="start of each record's third chunk (default: half the record)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    n, L = a.records, a.len
    key_len = 16 if "128" in a.aead else 32
    nl = 24 if a.aead.startswith("xchacha") else 12
    g = torch.Generator(device=dev).manual_seed(1)
    # chunk layout: record i occupies [base_i, base_i + L + 1) with a 1-byte
    # gap, so record starts (and most chunk starts) are unaligned
    sin, sout = L + a.in_gap, L + a.out_gap
    src = torch.randint(0, 256, (n * sin + 64,), dtype=torch.uint8, device=dev, generator=g)
    dst = torch.zeros(n * sout + 64, dtype=torch.uint8, device=dev)
    bin_ = torch.arange(n, dtype=torch.int64, device=dev) * sin
    bout = torch.arange(n, dtype=torch.int64, device=dev) * sout
    cut1 = torch.full((n,), min(a.cut1, L), dtype=torch.int64, device=dev)
    c2 = L // 2 if a.cut2 < 0 else min(a.cut2, L)
    cut2 = torch.full((n,), max(min(a.cut1, L), c2), dtype=torch.int64, device=dev)
    offs = torch.stack([torch.zeros_like(cut1), cut1, cut2], 1)       # chunk start in record
    lens = torch.stack([cut1, cut2 - cut1, L - cut2], 1)              # chunk length
    iov = torch.stack([dst.data_ptr() + bout[:, None] + offs,
                       src.data_ptr() + bin_[:, None] + offs, lens], 2).reshape(-1, 3).contiguous()
    starts = torch.arange(0, 3 * n + 1, 3, dtype=torch.int64, device=dev)
    ad = torch.randint(0, 256, (13 * n,), dtype=torch.uint8, device=dev, generator=g)
    aiv = torch.stack([ad.data_ptr() + 13 * torch.arange(n, dtype=torch.int64, device=dev),
                       torch.full((n,), 13, dtype=torch.int64, device=dev)], 1).contiguous()
    astarts = torch.arange(0, n + 1, dtype=torch.int64, device=dev)
    nonces = torch.randint(0, 256, (nl * n,), dtype=torch.uint8, device=dev, generator=g)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    ctx = ba.AEADCtx(a.aead, bytes(range(key_len)), 16)
    b = ba.make_iov_batch(n, iov, starts, tags, nonces, nl, aadvecs=aiv, aadvec_start=astarts,
                          status=status)
    # The same records, contiguous and 16-byte aligned, for comparison.
    cpt = torch.randint(0, 256, (n * ((L + 15) // 16 * 16) + 16,), dtype=torch.uint8, device=dev,
                        generator=g)
    cct = torch.zeros_like(cpt)
    cb = ba.make_batch(n, cpt, cct, tags, nonces, nl, ad, record_stride=(L + 15) // 16 * 16,
                       record_len=L, ad_stride=13, ad_len=13, status=status)
    # ... and contiguous at the iovec layout's input stride (unaligned records
    # when in_gap is not a multiple of 16; in place).
    ub = ba.make_batch(n, src, src, tags, nonces, nl, ad, record_stride=sin, record_len=L,
                       ad_stride=13, ad_len=13, status=status)
    # ... and at that stride into the second arena (as the iovec batch writes).
    ub2 = ba.make_batch(n, src, dst, tags, nonces, nl, ad, record_stride=sin, record_len=L,
                        ad_stride=13, ad_len=13, status=status) if sin == sout else None
    # The iovec batch in place (every chunk's output = its input).
    iov_ip = iov.clone()
    iov_ip[:, 0] = iov_ip[:, 1]
    bip = ba.make_iov_batch(n, iov_ip, starts, tags, nonces, nl, aadvecs=aiv,
                            aadvec_start=astarts, status=status)
    res = {}
    runs = [("iovec", ctx.sealv_batch_device, b), ("iovec_in_place", ctx.sealv_batch_device, bip),
            ("contiguous", ctx.seal_batch_device, cb),
            ("contiguous_at_stride", ctx.seal_batch_device, ub)]
    if ub2 is not None:
        runs.append(("contiguous_at_stride_two_arenas", ctx.seal_batch_device, ub2))
    for name, op, batch in runs:
        op(batch)
        torch.cuda.synchronize()
        assert bool(status.all()), name
        t0 = time.perf_counter()
        for _ in range(a.steps):
            op(batch)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        res[name] = {"ms_per_batch": round(dt * 1e3, 3), "gib_per_s": round(n * L / dt / 2**30, 2)}
    print(json.dumps({"aead": a.aead, "records": n, "record_bytes": L, "in_gap": a.in_gap,
                      "out_gap": a.out_gap, "cut1": a.cut1, "cut2": int(cut2[0]), "chunks_per_record": 3, **res}))


if __name__ == "__main__":
    main()
