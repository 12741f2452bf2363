"""CPU checks of the generated sources of the table-free AES (no GPU):
`gcm_bs_io.inc` is exactly what tools/gen_bs_asm.py emits; `bs_sbox.inc`
(the 82 v_bitop3 LUTs of the bitsliced engine) and `sbox_portable.inc` (the
Boyar-Peralta gates of the key setup) are parsed and evaluated on all 256
inputs against the S-box definition (FIPS-197 5.1.1)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "boringssl_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools", "sbox"))

from bp_circuit import sbox_ref  # noqa: E402


def test_output_pass_inc_is_generated():
    env = {k: v for k, v in os.environ.items() if not k.startswith("BS_")}
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "gen_bs_asm.py")],
                                  env=env, text=True)
    assert out == open(os.path.join(CSRC, "gcm_bs_io.inc")).read()


def _eval_lut_inc(text, x):
    env = {f"in[{b}]": (x >> b) & 1 for b in range(8)}
    outs = {}
    for line in text.splitlines():
        m = re.match(r"\s*const uint32_t (\w+) = (in\[\d\]);", line)
        if m:
            env[m.group(1)] = env[m.group(2)]
            continue
        m = re.match(r"\s*const uint32_t (\w+) = __builtin_amdgcn_bitop3_b32\((\w+|0u), (\w+|0u), "
                     r"(\w+|0u), 0x([0-9a-f]+)\);", line)
        if m:
            a, b, c = (0 if v == "0u" else env[v] for v in m.group(2, 3, 4))
            tt = int(m.group(5), 16)
            env[m.group(1)] = (tt >> ((a << 2) | (b << 1) | c)) & 1  # v_bitop3: src0 is the MSB
            continue
        m = re.match(r"\s*out\[(\d)\] = (\w+);", line)
        if m:
            outs[int(m.group(1))] = env[m.group(2)]
    return sum(outs[b] << b for b in range(8))


def test_bitsliced_sbox_luts_exhaustive():
    text = open(os.path.join(CSRC, "bs_sbox.inc")).read()
    n = len(re.findall(r"__builtin_amdgcn_bitop3_b32", text))
    assert n == 82
    ref = sbox_ref()
    assert [_eval_lut_inc(text, x) for x in range(256)] == ref


def _eval_gate_inc(text, x):
    env = {f"in[{b}]": (x >> b) & 1 for b in range(8)}
    outs = {}
    for line in text.splitlines():
        m = re.match(r"\s*const uint32_t (\w+) = (.+);", line)
        if m:
            expr = m.group(2)
            if expr.startswith("in["):
                env[m.group(1)] = env[expr]
                continue
            m2 = re.match(r"~\((\w+) \^ (\w+)\)$", expr)
            if m2:
                env[m.group(1)] = 1 ^ env[m2.group(1)] ^ env[m2.group(2)]
                continue
            a, op, b = expr.split()
            env[m.group(1)] = env[a] ^ env[b] if op == "^" else env[a] & env[b]
            continue
        m = re.match(r"\s*out\[(\d)\] = (\w+);", line)
        if m:
            outs[int(m.group(1))] = env[m.group(2)]
    return sum(outs[b] << b for b in range(8))


def test_portable_sbox_gates_exhaustive():
    text = open(os.path.join(CSRC, "sbox_portable.inc")).read()
    assert [_eval_gate_inc(text, x) for x in range(256)] == sbox_ref()
