#!/usr/bin/env python3
"""Single-record latency of the host-buffer EVP_AEAD surface.

What an unbatched caller such as SSLAEADContext::SealScatter
(ssl/ssl_aead_ctx.cc:299-409) pays per record: EVP_AEAD_CTX_seal_scatter with
host buffers = copy in, prologue + bulk kernel, copy out, stream sync.
Prints one JSON object: median / p90 microseconds per call, and the same
calls on the reference CPU path (oracle/_ref/ref_tool bench1, one core).
"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import boringssl_amd as ba  # noqa: E402

L = ba.lib


def measure(aead, size, n=500):
    a = ba.EVP_aead(aead)
    ctx = ba.EVP_AEAD_CTX()
    key = bytes(L.EVP_AEAD_key_length(a))
    assert L.EVP_AEAD_CTX_init(ctypes.byref(ctx), a, key, len(key), 0, None)
    out = ctypes.create_string_buffer(size + 1)
    tag = ctypes.create_string_buffer(16)
    pt, ad, nonce = bytes(size), bytes(13), bytes(12)
    tl = ctypes.c_size_t(0)
    ts = []
    for i in range(n + 50):
        t0 = time.perf_counter()
        ok = L.EVP_AEAD_CTX_seal_scatter(ctypes.byref(ctx), out, tag, ctypes.byref(tl), 16, nonce,
                                         12, pt, size, None, 0, ad, 13)
        t1 = time.perf_counter()
        assert ok
        if i >= 50:
            ts.append(t1 - t0)
    L.EVP_AEAD_CTX_cleanup(ctypes.byref(ctx))
    ts.sort()
    return {"median_us": round(ts[len(ts) // 2] * 1e6, 1),
            "p90_us": round(ts[int(len(ts) * 0.9)] * 1e6, 1)}


def cpu_ref(aead, size):
    tool = os.path.join(ROOT, "oracle", "_ref", "ref_tool")
    if not os.path.exists(tool):
        return None
    r = json.loads(subprocess.check_output([tool, "bench1", aead, "seal", str(size), "1"],
                                           text=True))
    return round(r["seconds"] / r["iterations"] * 1e6, 3)


def main():
    import torch
    torch.cuda.set_device(0)
    res = {}
    for aead in ("aes-128-gcm", "chacha20-poly1305"):
        for size in (1350, 16384):
            r = measure(aead, size)
            r["reference_cpu_us"] = cpu_ref(aead, size)
            res[f"{aead}/{size}"] = r
    print(json.dumps({"single_record_seal_scatter_latency": res}))


if __name__ == "__main__":
    main()
