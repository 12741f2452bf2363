"""Fixture loading and the batch-digest definition shared by the CPU and GPU
parity tests (mirrors ref_tool.cc cmd_digest: tags_sha256 = SHA-256 over all
tags in record order; ct_sha256 = SHA-256 over the per-1024-record SHA-256 of
the concatenated ciphertexts)."""
import hashlib
import json
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

AEAD_KEYLEN = {"aes-128-gcm": 16, "aes-192-gcm": 24, "aes-256-gcm": 32, "chacha20-poly1305": 32,
               "xchacha20-poly1305": 32, "aes-128-gcm-siv": 16, "aes-256-gcm-siv": 32}


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def digest_chunks(ct_chunk_fn, nchunks, threads=16):
    """ct_chunk_fn(c) -> bytes-like of the concatenated ciphertexts of chunk c."""
    def one(c):
        return hashlib.sha256(ct_chunk_fn(c)).digest()
    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(one, range(nchunks)))
    return hashlib.sha256(b"".join(parts)).hexdigest()


def batch_digests(out, offsets, lens, tags, chunk=1024):
    """out: uint8 numpy array holding records at offsets (lengths lens)."""
    n = len(lens)
    nchunks = (n + chunk - 1) // chunk

    def chunk_bytes(c):
        lo, hi = c * chunk, min(n, (c + 1) * chunk)
        parts = [out[int(offsets[i]):int(offsets[i]) + int(lens[i])] for i in range(lo, hi)]
        return np.concatenate(parts).tobytes() if parts else b""

    ct = digest_chunks(chunk_bytes, nchunks)
    return hashlib.sha256(np.ascontiguousarray(tags).tobytes()).hexdigest(), ct
