#!/usr/bin/env python3
"""Diagnostic: do the T-table kernel (8-wave workgroups) and the bitsliced
kernel run side by side on the same CUs, and what does that buy?  Splits a
config-2 batch (AES-128-GCM, 16 KiB records) into a T-table part and a
bitsliced part launched on two streams; prints per-mode GiB/s and checks the
concurrent outputs against a single-kernel run.  Kernel choice per launch is
by environment (BSSL_AMD_GCM_BS / BSSL_AMD_GCM_W8), read at launch time."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import boringssl_amd as ba  # noqa: E402
from bench import synth_key  # noqa: E402


def sub_batch(t, lo, hi, L):
    pt, ct, tags, nonce, ad, st = t
    return ba.make_batch(hi - lo, pt[lo * L:], ct[lo * L:], tags[16 * lo:], nonce[12 * lo:], 12,
                         ad[13 * lo:], record_stride=L, record_len=L, ad_stride=13, ad_len=13,
                         status=st[lo:])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    L = 16384
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    import numpy as np
    offs = torch.from_numpy((np.arange(n, dtype=np.int64) * L)).to(dev)
    lens = torch.full((n,), L, dtype=torch.int64, device=dev)
    pt = torch.empty(n * L, dtype=torch.uint8, device=dev)
    ct = torch.empty_like(pt)
    nonce = torch.empty(12 * n, dtype=torch.uint8, device=dev)
    ad = torch.empty(13 * n, dtype=torch.uint8, device=dev)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.uint8, device=dev)
    ba.synth_fill_device(0, n, offs, lens, pt, nonce, ad)
    t = (pt, ct, tags, nonce, ad, st)
    ctx = ba.AEADCtx("aes-128-gcm", synth_key(0, 16), 16)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()

    def run(mode, frac, steps=6):
        na = int(n * frac) // 64 * 64
        A, B = sub_batch(t, 0, na, L), sub_batch(t, na, n, L)
        torch.cuda.synchronize()
        times = []
        for it in range(steps + 1):
            t0 = time.perf_counter()
            if mode in ("tt16", "tt8", "mix", "mix16"):
                os.environ["BSSL_AMD_GCM_BS"] = "0"
                os.environ["BSSL_AMD_GCM_W8"] = "0" if mode in ("tt16", "mix16") else "1"
                if na:
                    ctx.seal_batch_device(A, s1)
            if mode in ("bs", "mix", "mix16"):
                os.environ["BSSL_AMD_GCM_BS"] = "1"
                if na < n:
                    ctx.seal_batch_device(B, s2 if mode.startswith("mix") else s1)
            torch.cuda.synchronize()
            if it:
                times.append(time.perf_counter() - t0)
        os.environ["BSSL_AMD_GCM_BS"] = "0"
        os.environ["BSSL_AMD_GCM_W8"] = "0"
        dt = sorted(times)[len(times) // 2]
        done = (na if mode in ("tt16", "tt8") else n if mode.startswith("mix") else n - na)
        return done * L / dt / 2**30

    # reference output: T-table only
    print("tt16 all:", round(run("tt16", 1.0), 1), flush=True)
    ref_ct = ct[: 64 * L].clone()
    ref_tags = tags.clone()
    print("tt8 all:", round(run("tt8", 1.0), 1), flush=True)
    print("bs all:", round(run("bs", 0.0), 1), flush=True)
    tags.zero_()
    for f in (0.9, 0.8, 0.7, 0.6):
        g = run("mix", f)
        ok = torch.equal(tags, ref_tags) and bool(st.all())
        print(f"mix T8 {f:.1f} / bs {1-f:.1f}: {g:.1f} GiB/s  outputs_equal={ok}", flush=True)
        tags.zero_()
    for f in (0.85, 0.7):
        g = run("mix16", f)
        ok = torch.equal(tags, ref_tags) and bool(st.all())
        print(f"mix T16 {f:.2f} / bs: {g:.1f} GiB/s  outputs_equal={ok}", flush=True)
        tags.zero_()
    assert torch.equal(ct[: 64 * L], ref_ct)


if __name__ == "__main__":
    main()
