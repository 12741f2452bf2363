#!/usr/bin/env python3
"""Regenerates the committed fixtures under tests/golden/.

Run in the build container (where /root/reference exists); the GPU box only
reads the committed JSON.  Three kinds of fixture are produced:

* kat_*.json      -- the reference's OWN known-answer data, converted (not
                     copied: re-encoded as JSON records) from
                       crypto/cipher/test/aes_{128,192,256}_gcm_tests.txt
                       crypto/cipher/test/chacha20_poly1305_tests.txt
                       crypto/cipher/test/xchacha20_poly1305_tests.txt
                       crypto/cipher/test/aes_{128,256}_gcm_siv_tests.txt
                       third_party/wycheproof_testvectors/aes_gcm_test.txt
                       third_party/wycheproof_testvectors/chacha20_poly1305_test.txt
                       third_party/wycheproof_testvectors/xchacha20_poly1305_test.txt
                       third_party/wycheproof_testvectors/aes_gcm_siv_test.txt
                       crypto/fipsmodule/aes/aes_tests.txt
                       crypto/poly1305/poly1305_tests.txt
                     The field semantics follow crypto/cipher/aead_test.cc:188-281
                     (TestVector: tag_len = len(TAG)) and :1493-1564
                     (RunWycheproofTestCase: tagSize instruction, result).
* ref_edge.json   -- edge-case records sealed by the reference library built
                     from source into oracle/_ref/ (oracle/ref/Makefile):
                     `oracle/_ref/ref_tool edge`.
* ref_digests.json-- batch digests of the synthetic workloads of SURVEY.md
                     section 8(d) sealed by the reference library:
                     `oracle/_ref/ref_tool digest ...`.
* ref_shard_digests.json -- the same digests for every rank's shard of
                     `bench.py --gpus N` (N = 2, 4, 8; bench.shard_plan) of the
                     bench configs: `oracle/_ref/ref_tool shard ...`, so every
                     rank of a multi-GPU run is checked bit for bit (SURVEY.md
                     8(e): per-GPU digests, combined in a fixed order).

Usage: python tests/golden/make_golden.py [--skip-full] [--shards]
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("BSSL_REFERENCE", "/root/reference")
REF_TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_tool")


def parse_filetest(path):
    """Minimal reader for the reference FileTest format (KEY: value blocks,
    '[instr = v]' instruction lines, blank-line separated)."""
    cases, cur, instr = [], {}, {}
    with open(path) as f:
        for raw in f:
            line = raw.strip()
            if line.startswith("#"):
                continue
            if not line:
                if cur:
                    cur["_instr"] = dict(instr)
                    cases.append(cur)
                    cur = {}
                continue
            if line.startswith("[") and line.endswith("]"):
                if cur:
                    cur["_instr"] = dict(instr)
                    cases.append(cur)
                    cur = {}
                k, _, v = line[1:-1].partition("=")
                instr[k.strip()] = v.strip()
                continue
            if ":" in line and (line.split(":")[0].isupper() or line.split(":")[0][:1].isupper()):
                k, _, v = line.partition(":")
            else:
                k, _, v = line.partition("=")
            cur[k.strip()] = v.strip()
    if cur:
        cur["_instr"] = dict(instr)
        cases.append(cur)
    return cases


def unq(v):
    v = v.strip()
    if v.startswith('"') and v.endswith('"'):
        return v[1:-1].encode().hex()
    return v


def convert_aead():
    out = []
    files = [
        ("crypto/cipher/test/aes_128_gcm_tests.txt", "aes-128-gcm"),
        ("crypto/cipher/test/aes_192_gcm_tests.txt", "aes-192-gcm"),
        ("crypto/cipher/test/aes_256_gcm_tests.txt", "aes-256-gcm"),
        ("crypto/cipher/test/chacha20_poly1305_tests.txt", "chacha20-poly1305"),
        ("crypto/cipher/test/xchacha20_poly1305_tests.txt", "xchacha20-poly1305"),
        ("crypto/cipher/test/aes_128_gcm_siv_tests.txt", "aes-128-gcm-siv"),
        ("crypto/cipher/test/aes_256_gcm_siv_tests.txt", "aes-256-gcm-siv"),
    ]
    for rel, aead in files:
        for i, c in enumerate(parse_filetest(os.path.join(REF, rel))):
            out.append({
                "source": f"{rel}#{i}", "aead": aead, "key": unq(c["KEY"]),
                "nonce": unq(c["NONCE"]), "ad": unq(c["AD"]), "pt": unq(c["IN"]),
                "ct": unq(c["CT"]), "tag": unq(c["TAG"]), "valid": True,
            })
    wfiles = [
        ("third_party/wycheproof_testvectors/aes_gcm_test.txt", "gcm"),
        ("third_party/wycheproof_testvectors/chacha20_poly1305_test.txt", "chacha"),
        ("third_party/wycheproof_testvectors/xchacha20_poly1305_test.txt", "xchacha"),
        ("third_party/wycheproof_testvectors/aes_gcm_siv_test.txt", "siv"),
    ]
    for rel, kind in wfiles:
        for c in parse_filetest(os.path.join(REF, rel)):
            ins = c["_instr"]
            if kind == "gcm":
                aead = {"128": "aes-128-gcm", "192": "aes-192-gcm", "256": "aes-256-gcm"}[ins["keySize"]]
            elif kind == "siv":
                aead = {"128": "aes-128-gcm-siv", "256": "aes-256-gcm-siv"}.get(ins["keySize"])
                if aead is None:
                    continue  # 192-bit keys: no such EVP_AEAD
            elif kind == "chacha":
                aead = "chacha20-poly1305"
            else:
                aead = "xchacha20-poly1305"
            tag_len = int(ins["tagSize"]) // 8
            out.append({
                "source": f"{rel}#tcId={c.get('tcId', '?')}", "aead": aead, "key": c["key"],
                "nonce": c["iv"], "ad": c["aad"], "pt": c["msg"], "ct": c["ct"],
                "tag": c["tag"], "tag_len": tag_len, "valid": c["result"] == "valid",
                "flags": c.get("flags", ""),
            })
    return out


def _tcids(path):
    ids = []
    with open(path) as f:
        for line in f:
            if line.startswith("# tcId"):
                ids.append(line.split("=")[1].strip())
    return ids


def convert_aes():
    out = []
    for i, c in enumerate(parse_filetest(os.path.join(REF, "crypto/fipsmodule/aes/aes_tests.txt"))):
        out.append({"source": f"crypto/fipsmodule/aes/aes_tests.txt#{i}", "mode": c["Mode"],
                    "key": c["Key"], "pt": c["Plaintext"], "ct": c["Ciphertext"]})
    return out


def convert_poly():
    out = []
    for i, c in enumerate(parse_filetest(os.path.join(REF, "crypto/poly1305/poly1305_tests.txt"))):
        out.append({"source": f"crypto/poly1305/poly1305_tests.txt#{i}", "key": unq(c["Key"]),
                    "input": unq(c["Input"]), "mac": unq(c["MAC"])})
    return out


# Batch-digest workloads; "parity" sizes are checked in full by
# the GPU tests, "config" sizes are the BASELINE.json configs themselves.
DIGESTS = [
    ("parity_aes128_16k", "aes-128-gcm", 1, 4096, "16384"),
    ("parity_aes256_mixed", "aes-256-gcm", 1, 8192, "mixed"),
    ("parity_chacha_1350", "chacha20-poly1305", 1, 16384, "1350"),
    ("parity_multikey_aes128", "aes-128-gcm", 256, 16, "16384"),
    ("parity_xchacha_1350", "xchacha20-poly1305", 1, 16384, "1350"),
    ("parity_siv128_1350", "aes-128-gcm-siv", 1, 16384, "1350"),
    ("parity_siv256_mixed", "aes-256-gcm-siv", 1, 4096, "mixed"),
    ("parity_siv128_multikey", "aes-128-gcm-siv", 64, 16, "16384"),
    ("config2_aes128_16k", "aes-128-gcm", 1, 1048576, "16384"),
    ("config3_chacha_1350", "chacha20-poly1305", 1, 1048576, "1350"),
    ("config3x_xchacha_1350", "xchacha20-poly1305", 1, 1048576, "1350"),
    # bench.py --config configG (AES-128-GCM on config 3's records; round 3)
    ("configG_aes128_1350", "aes-128-gcm", 1, 1048576, "1350"),
    ("configs_siv128_16k", "aes-128-gcm-siv", 1, 262144, "16384"),
    # bench.py --config configS's own batch (1M records; round 3)
    ("configS_siv128_16k_1m", "aes-128-gcm-siv", 1, 1048576, "16384"),
    ("config4_aes256_mixed", "aes-256-gcm", 1, 4194304, "mixed"),
    ("config5_multikey_aes128", "aes-128-gcm", 65536, 64, "16384"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only", default="", help="regenerate just this digest entry")
    ap.add_argument("--tls-only", action="store_true", help="regenerate ref_tls.json only")
    ap.add_argument("--shards", action="store_true",
                    help="(re)generate ref_shard_digests.json only")
    args = ap.parse_args()
    if args.shards:
        return shard_entries()
    if args.tls_only:
        return write_ref_tls()
    if args.only:
        return digest_entries(lambda name: name == args.only)
    aead = convert_aead()
    # attach Wycheproof tcIds (comment lines precede each record in file order)
    for rel in ("third_party/wycheproof_testvectors/aes_gcm_test.txt",
                "third_party/wycheproof_testvectors/chacha20_poly1305_test.txt",
                "third_party/wycheproof_testvectors/xchacha20_poly1305_test.txt",
                "third_party/wycheproof_testvectors/aes_gcm_siv_test.txt"):
        ids = _tcids(os.path.join(REF, rel))
        recs = [r for r in aead if r["source"].startswith(rel)]
        assert len(ids) == len(recs), (rel, len(ids), len(recs))
        for r, t in zip(recs, ids):
            r["source"] = f"{rel}#tcId={t}"
    with open(os.path.join(HERE, "kat_aead.json"), "w") as f:
        json.dump(aead, f, indent=0)
    with open(os.path.join(HERE, "kat_aes.json"), "w") as f:
        json.dump(convert_aes(), f, indent=0)
    with open(os.path.join(HERE, "kat_poly1305.json"), "w") as f:
        json.dump(convert_poly(), f, indent=0)
    print(f"kat_aead.json: {len(aead)} cases")

    if not os.path.exists(REF_TOOL):
        subprocess.check_call(["make", "-j8", "-C", os.path.join(ROOT, "oracle", "ref")])
    edge = json.loads(subprocess.check_output([REF_TOOL, "edge"]))
    with open(os.path.join(HERE, "ref_edge.json"), "w") as f:
        json.dump(edge, f, indent=0)
    print(f"ref_edge.json: {len(edge)} cases")

    write_ref_tls()
    return digest_entries(lambda name: not (args.skip_full and name.startswith("config")))


def write_ref_tls():
    """ref_tls.json: TLS 1.2/1.3 records sealed by the reference's own
    SSLAEADContext (oracle/_ref/ref_tls, built from /root/reference/ssl)."""
    tool = os.path.join(ROOT, "oracle", "_ref", "ref_tls")
    if not os.path.exists(tool):
        subprocess.check_call(["make", "-j8", "-C", os.path.join(ROOT, "oracle", "ref")])
    recs = json.loads(subprocess.check_output([tool]))
    with open(os.path.join(HERE, "ref_tls.json"), "w") as f:
        json.dump(recs, f, indent=0)
    print(f"ref_tls.json: {sum(len(r['records']) for r in recs)} records")


def digest_entries(want):
    if not os.path.exists(REF_TOOL):
        subprocess.check_call(["make", "-j8", "-C", os.path.join(ROOT, "oracle", "ref")])
    path = os.path.join(HERE, "ref_digests.json")
    digests = {}
    if os.path.exists(path):
        with open(path) as f:
            digests = json.load(f)
    for name, aead_name, nkeys, rpk, length in DIGESTS:
        if not want(name):
            continue
        res = json.loads(subprocess.check_output(
            [REF_TOOL, "digest", aead_name, str(nkeys), str(rpk), length, "8"]))
        digests[name] = res
        print(name, res["tags_sha256"][:16], res["ct_sha256"][:16], flush=True)
        with open(path, "w") as f:
            json.dump(digests, f, indent=1, sort_keys=True)


# bench.py configs whose multi-GPU shards get reference digests, and the GPU
# counts of the driver's scaling run.
SHARD_CONFIGS = ["config2", "config3", "config3x", "configG", "configS", "config4", "config5"]
SHARD_WORLDS = [2, 4, 8]


def shard_key(aead, length, first, n, rpk):
    """Identity of a shard digest: records [first, first + n) of the synthetic
    sequence, key i // rpk (rpk 0: one key), lengths `length` or "mixed"."""
    return f"{aead}/{length}/first={first}/n={n}/rpk={rpk}"


def bench_shards():
    """(key, aead, length, first, n, rpk, [(config, world, rank), ...]) for
    every rank's shard of bench.py --gpus N, N in SHARD_WORLDS."""
    sys.path.insert(0, ROOT)
    import bench
    shards = {}
    for config in SHARD_CONFIGS:
        aead, _, _, length, _, _ = bench.CONFIGS[config]
        rpk = bench.RECORDS_PER_KEY.get(config, 0)
        for world in SHARD_WORLDS:
            for rank in range(world):
                sh = bench.shard_plan(config, rank, world)
                key = shard_key(aead, length, sh.first, sh.n, rpk)
                ent = shards.setdefault(key, [key, aead, str(length), sh.first, sh.n, rpk, []])
                ent[6].append((config, world, rank))
    return list(shards.values())


# Small shards at a non-zero first record (and key), checked against the CPU
# oracle by tests/test_shard_digests.py: they pin the shard definition that
# the multi-GPU digests above use.
PIN_SHARDS = [
    ("aes-128-gcm", "16384", 320, 192, 64),
    ("aes-256-gcm", "mixed", 1000, 3000, 0),
    ("chacha20-poly1305", "1350", 5000, 2048, 0),
    ("xchacha20-poly1305", "1350", 7, 1500, 0),
    ("aes-128-gcm-siv", "16384", 1100, 300, 0),
]


def shard_entries():
    if not os.path.exists(REF_TOOL):
        subprocess.check_call(["make", "-j8", "-C", os.path.join(ROOT, "oracle", "ref")])
    path = os.path.join(HERE, "ref_shard_digests.json")
    digests = {}
    if os.path.exists(path):
        with open(path) as f:
            digests = json.load(f)
    for key, aead, length, first, n, rpk, users in bench_shards():
        if key in digests:
            continue
        res = json.loads(subprocess.check_output(
            [REF_TOOL, "shard", aead, length, str(first), str(n), str(rpk), "8"]))
        res["used_by"] = [f"{c} N={w} rank {r}" for c, w, r in users]
        digests[key] = res
        print(key, res["tags_sha256"][:16], res["ct_sha256"][:16], flush=True)
        with open(path, "w") as f:
            json.dump(digests, f, indent=1, sort_keys=True)
    for aead, length, first, n, rpk in PIN_SHARDS:
        key = shard_key(aead, length, first, n, rpk)
        if key in digests:
            continue
        res = json.loads(subprocess.check_output(
            [REF_TOOL, "shard", aead, length, str(first), str(n), str(rpk), "8"]))
        res["used_by"] = ["tests/test_shard_digests.py (oracle pin)"]
        digests[key] = res
        with open(path, "w") as f:
            json.dump(digests, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    sys.exit(main())
