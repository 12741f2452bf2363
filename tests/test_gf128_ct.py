"""The constant-time GHASH multiply of the product (boringssl_amd/csrc/gf128_ct.h,
integer multiplication with holes -- the technique of the reference's
crypto/fipsmodule/aes/gcm_nohw.cc.inc:38-82) compiled for the host and
checked against the oracle's bitwise SP 800-38D multiply (oracle_gf128_mul):
random operands, sparse and dense edge values, and the gf_prep step.  CPU
only; the GPU tests cover the same header through the kernels."""
import ctypes
import os
import random
import subprocess

import pytest

import oracle_lib as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include "gf128_ct.h"
using namespace bssl_amd;
extern "C" void gf_mul_bytes(const uint8_t *x, const uint8_t *h, uint8_t *out) {
  gf_to_bytes(gf_mul(gf_from_bytes(x), gf_prep(gf_from_bytes(h))), out);
}
extern "C" unsigned long long clmul32_c(unsigned a, unsigned b) { return clmul32(a, b); }
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("gf")
    src, so = d / "gf.cc", d / "libgf.so"
    src.write_text(SRC)
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17",
                           "-I", os.path.join(ROOT, "boringssl_amd", "csrc"), str(src),
                           "-o", str(so)])
    lib = ctypes.CDLL(str(so))
    lib.clmul32_c.restype = ctypes.c_ulonglong
    lib.clmul32_c.argtypes = [ctypes.c_uint, ctypes.c_uint]
    return lib


def _clmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        b >>= 1
    return r


def test_clmul32(lib):
    rng = random.Random(1)
    vals = [0, 1, 0xffffffff, 0x80000000, 0x11111111, 0xeeeeeeee, 0xaaaaaaaa]
    vals += [rng.getrandbits(32) for _ in range(300)]
    for a in vals:
        for b in vals[:40]:
            assert lib.clmul32_c(a, b) == _clmul(a, b), (hex(a), hex(b))


def test_gf_mul_vs_oracle(lib):
    rng = random.Random(2)
    edge = [bytes(16), bytes([0x80]) + bytes(15), bytes(15) + b"\x01", b"\xff" * 16,
            bytes(15) + b"\x80", b"\x01" + bytes(15)]
    xs = edge + [rng.randbytes(16) for _ in range(400)]
    out = ctypes.create_string_buffer(16)
    for i, x in enumerate(xs):
        h = xs[(i * 7 + 3) % len(xs)] if i % 3 else rng.randbytes(16)
        lib.gf_mul_bytes(x, h, out)
        assert out.raw == o.gf128_mul(x, h), (x.hex(), h.hex())
    for x in edge:
        for h in edge:
            lib.gf_mul_bytes(x, h, out)
            assert out.raw == o.gf128_mul(x, h), (x.hex(), h.hex())
