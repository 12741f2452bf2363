#!/usr/bin/env python3
"""Diagnostic: config 2 (AES-128-GCM, 1M x 16 KiB) with each GCM kernel mode
(BSSL_AMD_GCM_MODE = table | bs | hybrid): GiB/s, bulk-kernel ms, and the
outputs of every mode against the table mode's."""
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
    n = int(os.environ.get("N", 1 << 20))
    L = int(os.environ.get("LEN", 16384))
    aead = os.environ.get("AEAD", "aes-128-gcm")
    modes = sys.argv[1:] or ["table", "mix4", "mix8", "bs", "hybrid"]
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
    ctx = ba.AEADCtx(aead, synth_key(0, 32 if "256" in aead else 16), 16)
    ref = None
    for mode in modes:
        os.environ["BSSL_AMD_GCM_MODE"] = mode
        tags.zero_()
        st.zero_()
        ctx.seal_batch_device(b)
        torch.cuda.synchronize()
        ba.set_kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(10):
            ctx.seal_batch_device(b)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        km = ba.collect_kernel_times()
        ba.set_kernel_timing(False)
        h = (tags.clone(), ct[:1 << 24].clone(), ct[-(1 << 24):].clone())
        if ref is None:
            ref = h
        ok = all(torch.equal(x, y) for x, y in zip(h, ref)) and bool(st.all())
        print(f"{mode:7s}: {n * L / dt / 2**30:8.1f} GiB/s  kernel {np.median(km):.3f} ms "
              f"(min {min(km):.3f})  equal={ok}", flush=True)


if __name__ == "__main__":
    main()
