#!/usr/bin/env python3
"""Per-key setup cost: EVP_AEAD_CTX_init + _cleanup of one
AES-GCM key (host tables + device copy), BSSL_AMD_KEYSET_new of config 5's
65,536 keys (device key-setup kernel) and, for comparison, the same tables
built by the host path.  Prints one JSON line.  Usage: python3
tools/keysetup_bench.py [--keys 65536]"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import boringssl_amd as ba  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=int, default=65536)
ap.add_argument("--init-reps", type=int, default=300)
a = ap.parse_args()
L = ba.lib
res = {}


def say(*x):
    print(*x, file=sys.stderr, flush=True)


for name, kl in (("aes-128-gcm", 16), ("aes-256-gcm", 32)):
    aead = ba.EVP_aead(name)
    key = bytes(range(kl))
    ctx = ba.EVP_AEAD_CTX()
    for _ in range(20):  # warm-up (first hipMalloc, module load)
        L.EVP_AEAD_CTX_zero(ctypes.byref(ctx))
        assert L.EVP_AEAD_CTX_init(ctypes.byref(ctx), aead, key, kl, 16, None)
        L.EVP_AEAD_CTX_cleanup(ctypes.byref(ctx))
    say(name, "warm")
    ti, tc = [], []
    for _ in range(a.init_reps):
        L.EVP_AEAD_CTX_zero(ctypes.byref(ctx))
        t0 = time.perf_counter()
        assert L.EVP_AEAD_CTX_init(ctypes.byref(ctx), aead, key, kl, 16, None)
        t1 = time.perf_counter()
        L.EVP_AEAD_CTX_cleanup(ctypes.byref(ctx))
        t2 = time.perf_counter()
        ti.append(t1 - t0)
        tc.append(t2 - t1)
    res[name] = {"ctx_init_us_median": round(statistics.median(ti) * 1e6, 1),
                 "ctx_init_us_p90": round(sorted(ti)[int(0.9 * len(ti))] * 1e6, 1),
                 "ctx_cleanup_us_median": round(statistics.median(tc) * 1e6, 1)}
    say(name, "ctx init done", res[name])
    keys = os.urandom(a.keys * kl)
    tk = []
    for _ in range(5):
        t0 = time.perf_counter()
        h = L.BSSL_AMD_KEYSET_new(aead, keys, a.keys, 16)
        t1 = time.perf_counter()
        assert h
        L.BSSL_AMD_KEYSET_free(h)
        tk.append(t1 - t0)
        say(name, "keyset", round((t1 - t0) * 1e3, 2), "ms")
    res[name]["keyset_new_ms_median"] = round(statistics.median(tk) * 1e3, 2)
    res[name]["keyset_new_ms_all"] = [round(x * 1e3, 2) for x in tk]
    n = min(a.keys, 16384)
    t0 = time.perf_counter()
    ba.gcm_key_tables(keys[:n * kl], kl, on_device=False)
    res[name]["host_tables_us_per_key"] = round((time.perf_counter() - t0) / n * 1e6, 2)
    t0 = time.perf_counter()
    ba.gcm_key_tables(keys[:n * kl], kl, on_device=True)
    res[name]["device_tables_plus_d2h_ms_%d_keys" % n] = round((time.perf_counter() - t0) * 1e3, 2)
print(json.dumps({"keys": a.keys, "results": res}))
