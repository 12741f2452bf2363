"""Generates tests/golden/gcm_key_tables.json: SHA-256 of the per-key device
tables (GcmKeyDev, internal.h) for 24 AES keys (16 / 24 / 32 bytes), as
computed by the round-4 host key setup (key_setup.cc at commit 52b6ea8: table
S-box scanned in constant time, bitwise GF(2^128) products).  The round-5 key
setup (key_sched.h, host and device) must reproduce every table byte for
byte.  Usage: python3 tools/golden/gen_key_tables.py HARNESS > json, where
HARNESS reads hex keys on stdin and writes the raw tables."""
import hashlib
import json
import random
import subprocess
import sys

SIZE = 12816
keys = []
rng = random.Random(20251018)
for kl in (16, 24, 32):
    keys += [bytes(kl), b"\xff" * kl, bytes(range(kl))]
    keys += [bytes(rng.randrange(256) for _ in range(kl)) for _ in range(5)]
out = subprocess.run([sys.argv[1]], input="".join(k.hex() + "\n" for k in keys).encode(),
                     capture_output=True, check=True).stdout
assert len(out) == SIZE * len(keys), len(out)
rows = [{"key": k.hex(), "sha256": hashlib.sha256(out[i * SIZE:(i + 1) * SIZE]).hexdigest()}
        for i, k in enumerate(keys)]
json.dump({"struct_bytes": SIZE, "source": "key_setup.cc @ 52b6ea8 (round-4 host key setup)",
           "tables": rows}, sys.stdout, indent=1)
print()
