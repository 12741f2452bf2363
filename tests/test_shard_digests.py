"""Reference digests for every rank of a multi-GPU bench run (CPU).

`bench.py --gpus N` seals one shard per rank (bench.shard_plan: weak configs
records [r*n, (r+1)*n), config 4 byte-balanced ranges of one 4M-record batch,
config 5 key ranges of one 64K-key set) and digests each rank's output
against tests/golden/ref_shard_digests.json, which the reference library
itself produced (oracle/_ref/ref_tool shard, tests/golden/make_golden.py
--shards).  These tests check, without a GPU, that

* every rank of every bench config at N = 2, 4, 8 has its digest, keyed the
  way bench.golden_entry looks it up;
* the shard command and the whole-workload command of ref_tool agree (rank 0
  of a weak config is the N = 1 workload of ref_digests.json);
* the shard definition (first record, per-record key i // rpk, global
  record index in nonce/AD/plaintext/length) is the oracle's: small shards at
  a non-zero first record, sealed by the CPU oracle, give the committed
  reference digests.
"""
import os
import sys
import types

import numpy as np
import pytest

import bench
import oracle_lib as o
from golden_util import AEAD_KEYLEN, batch_digests, load

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden  # noqa: E402

AEAD_ID = {"aes-128-gcm": o.AES_GCM, "aes-256-gcm": o.AES_GCM,
           "chacha20-poly1305": o.CHACHA20_POLY1305, "xchacha20-poly1305": o.XCHACHA20_POLY1305,
           "aes-128-gcm-siv": o.AES_GCM_SIV}


@pytest.fixture(scope="module")
def shards():
    return load("ref_shard_digests.json")


@pytest.mark.parametrize("config", make_golden.SHARD_CONFIGS)
@pytest.mark.parametrize("world", make_golden.SHARD_WORLDS)
def test_every_rank_has_a_reference_digest(shards, config, world):
    aead, _, _, length, _, _ = bench.CONFIGS[config]
    for rank in range(world):
        sh = bench.shard_plan(config, rank, world)
        w = types.SimpleNamespace(config=config, aead=aead, shard=sh, nrec=sh.n,
                                  nkeys=sh.nkeys or 1)
        ge = bench.golden_entry(w)
        assert ge is not None, (config, world, rank)
        name, g = ge
        assert name in shards
        assert g["aead"] == aead and g["first"] == sh.first and g["records"] == sh.n
        assert g["bytes"] == int(sh.lens.sum())
        assert g["records_per_key"] == bench.RECORDS_PER_KEY.get(config, 0)


def test_shard_command_agrees_with_whole_workload_digests(shards):
    full = load("ref_digests.json")
    pairs = [("config2_aes128_16k", "aes-128-gcm", "16384"),
             ("config3_chacha_1350", "chacha20-poly1305", "1350"),
             ("config3x_xchacha_1350", "xchacha20-poly1305", "1350"),
             ("configG_aes128_1350", "aes-128-gcm", "1350"),
             ("configS_siv128_16k_1m", "aes-128-gcm-siv", "16384")]
    for name, aead, length in pairs:
        s = shards[bench.shard_key(aead, length, 0, 1 << 20, 0)]
        assert (s["tags_sha256"], s["ct_sha256"]) == (full[name]["tags_sha256"],
                                                     full[name]["ct_sha256"]), name


def test_shards_cover_the_strong_batches(shards):
    """Config 4 / 5 shards of one N concatenate to the whole batch (tags of
    the first and last record agree with the N = 1 digest's)."""
    full = load("ref_digests.json")
    for config, name in (("config4", "config4_aes256_mixed"), ("config5", "config5_multikey_aes128")):
        for world in make_golden.SHARD_WORLDS:
            plan = [bench.shard_plan(config, r, world) for r in range(world)]
            rpk = bench.RECORDS_PER_KEY.get(config, 0)
            ents = [shards[bench.shard_key(bench.CONFIGS[config][0], bench.CONFIGS[config][3],
                                           p.first, p.n, rpk)] for p in plan]
            assert sum(e["records"] for e in ents) == full[name]["records"]
            assert sum(e["bytes"] for e in ents) == full[name]["bytes"]
            assert ents[0]["tag_first"] == full[name]["tag_first"]
            assert ents[-1]["tag_last"] == full[name]["tag_last"]


@pytest.mark.parametrize("aead,length,first,n,rpk", make_golden.PIN_SHARDS)
def test_oracle_matches_reference_shard_digest(shards, aead, length, first, n, rpk):
    g = shards[bench.shard_key(aead, length, first, n, rpk)]
    lens = (bench.mixed_lengths(first, n) if length == "mixed"
            else np.full(n, int(length), dtype=np.uint64))
    pt, offs, nonces, ads = o.synth_batch(first, lens)
    key_len = AEAD_KEYLEN[aead]
    if rpk:
        k0 = first // rpk
        nk = (first + n - 1) // rpk - k0 + 1
        keys = np.frombuffer(b"".join(o.synth_key(k0 + k, key_len) for k in range(nk)),
                             dtype=np.uint8).copy()
        kidx = ((np.arange(first, first + n, dtype=np.uint64) // np.uint64(rpk)) -
                np.uint64(k0)).astype(np.uint32)
    else:
        keys = np.frombuffer(o.synth_key(0, key_len), dtype=np.uint8).copy()
        kidx = None
    nl = 12
    if aead == "xchacha20-poly1305":
        nonces, nl = o.xchacha_nonces(nonces), 24
    out = np.zeros_like(pt)
    tags = np.zeros(16 * n, dtype=np.uint8)
    failed = o.batch(AEAD_ID[aead], 1, keys, key_len, kidx, pt, out, offs, lens, nonces, nl, ads,
                     np.arange(n, dtype=np.uint64) * np.uint64(13), np.full(n, 13, np.uint64),
                     tags, 16)
    assert failed == 0
    assert batch_digests(out, offs, lens, tags) == (g["tags_sha256"], g["ct_sha256"])
