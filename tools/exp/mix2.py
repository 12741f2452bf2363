#!/usr/bin/env python3
"""Diagnostic: BSSL_AMD_GCM_MIX=p splits a uniform 16 KiB batch inside the
launcher: p% of the records to the 8-wave T-table kernel on the caller's
stream and the rest to the bitsliced kernel on a second stream, after one
shared prologue.  Prints GiB/s per split and checks outputs."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import boringssl_amd as ba  # noqa: E402
from bench import synth_key  # noqa: E402


def main():
    n, L = 1 << 20, 16384
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    offs = torch.from_numpy(np.arange(n, dtype=np.int64) * L).to(dev)
    lens = torch.full((n,), L, dtype=torch.int64, device=dev)
    pt = torch.empty(n * L, dtype=torch.uint8, device=dev)
    ct = torch.empty_like(pt)
    nonce = torch.empty(12 * n, dtype=torch.uint8, device=dev)
    ad = torch.empty(13 * n, dtype=torch.uint8, device=dev)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    ba.synth_fill_device(0, n, offs, lens, pt, nonce, ad)
    b = ba.make_batch(n, pt, ct, tags, nonce, 12, ad, record_stride=L, record_len=L, ad_stride=13,
                      ad_len=13, status=st)
    ctx = ba.AEADCtx("aes-128-gcm", synth_key(0, 16), 16)
    ref = None
    for mix in [0] + [int(x) for x in (sys.argv[1:] or ["95", "90", "85", "80", "75", "70", "60"])]:
        os.environ["BSSL_AMD_GCM_MIX"] = str(mix)
        tags.zero_()
        ctx.seal_batch_device(b)
        torch.cuda.synchronize()
        ba.set_kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(8):
            ctx.seal_batch_device(b)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 8
        km = ba.collect_kernel_times()
        ba.set_kernel_timing(False)
        if ref is None:
            ref = (tags.clone(), ct[:1 << 24].clone(), ct[-(1 << 24):].clone())
        ok = (torch.equal(tags, ref[0]) and torch.equal(ct[:1 << 24], ref[1]) and
              torch.equal(ct[-(1 << 24):], ref[2]) and bool(st.all()))
        print(f"mix {mix:3d}: {n * L / dt / 2**30:7.1f} GiB/s  kernel {np.median(km):.3f} ms  "
              f"equal={ok}", flush=True)


if __name__ == "__main__":
    main()
