"""The table-free AES-GCM engine for every batch.

With the bitsliced engine selected (BSSL_AMD_set_aes_gcm_engine) every AES-GCM
batch runs on gcm_bs.hip (gcm_bs_kernel / gcm_bs_keyset_kernel; no AES table
in LDS or memory, north_star "no T-tables", reference
aes_nohw.cc.inc:508,866-878): one-key and keyset batches, any record length,
alignment and AD, extra bytes (the TLS 1.3 inner type), iovec records and
single records.  This module re-runs the GCM cases of the parity suite under
that engine, and the bench's own layouts of configs 2, 4, 5 and G at reduced
size against the reference library's digests or the CPU oracle.
"""
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import boringssl_amd as ba  # noqa: E402
import oracle_lib as o  # noqa: E402

import test_aead_api_gpu as api  # noqa: E402
import test_gpu_parity as par  # noqa: E402
import test_tls_golden as tlsg  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu
GCM = ["aes-128-gcm", "aes-256-gcm"]


@pytest.fixture(autouse=True)
def _bs16(aes_engine):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    aes_engine("bs")
    yield


@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-192-gcm", "aes-256-gcm"])
def test_kat_single_record(aead):
    par.test_kat_single_record(aead)


def test_ref_edge_single_record():
    par.test_ref_edge_single_record()


@pytest.mark.parametrize("source", ["ref_edge.json", "kat_aead.json"])
def test_batch_multikey_vectors(source):
    par.test_batch_multikey_vectors(source)


@pytest.mark.parametrize("aead", GCM)
@pytest.mark.parametrize("layout", ["aligned", "unaligned", "inplace"])
def test_batch_ragged_vs_oracle(aead, layout):
    par.test_batch_ragged_vs_oracle(aead, layout)


@pytest.mark.parametrize("aead", GCM)
@pytest.mark.parametrize("multikey", [False, True])
def test_batch_large_ragged_reordered(aead, multikey):
    par.test_batch_large_ragged_reordered(aead, multikey)


def test_batch_gcm_nonce_lengths_and_truncated_tags():
    par.test_batch_gcm_nonce_lengths_and_truncated_tags()


@pytest.mark.parametrize("aead", GCM)
def test_open_rejects_tampering_and_zeroes_output(aead):
    par.test_open_rejects_tampering_and_zeroes_output(aead)


@pytest.mark.parametrize("aead", GCM)
def test_iovec_batch_vs_oracle(aead):
    par.test_iovec_batch_vs_oracle(aead)


@pytest.mark.parametrize("aead", GCM)
@pytest.mark.parametrize("n", [300, 4500])
def test_iovec_in_place_walk(aead, n):
    par.test_iovec_in_place_walk(aead, n)


@pytest.mark.parametrize("version,aead", [(0x0303, "aes-128-gcm"), (0x0303, "aes-256-gcm"),
                                          (0x0304, "aes-128-gcm"), (0x0304, "aes-256-gcm")])
def test_tls_record_layer(version, aead):
    par.test_tls_record_layer(version, aead)


@pytest.mark.parametrize("case", [c for c in tlsg.CASES if "gcm" in c["aead"]],
                         ids=[i for c, i in zip(tlsg.CASES, tlsg.IDS) if "gcm" in c["aead"]])
def test_tls_shim_matches_reference(case):
    tlsg.test_tls_shim_matches_reference(case)


@pytest.mark.parametrize("aead", GCM)
def test_extra_input(aead):
    api.test_extra_input(aead)


@pytest.mark.parametrize("aead", GCM)
def test_truncated_tags(aead):
    api.test_truncated_tags(aead)


@pytest.mark.parametrize("aead", GCM)
@pytest.mark.parametrize("in_place", [False, True])
def test_sealv(aead, in_place):
    api.test_sealv(aead, in_place)


@pytest.mark.parametrize("aead", GCM)
@pytest.mark.parametrize("in_place", [False, True])
def test_openv_detached(aead, in_place):
    api.test_openv_detached(aead, in_place)


@pytest.mark.parametrize("aead", GCM)
def test_unaligned_input(aead):
    api.test_unaligned_input(aead)


# The bench's own layouts at reduced size (uniform 128-byte-aligned records
# with no per-record arrays for configs 2 and G, per-record offsets/lengths and
# the length-ordered schedule for config 4, a keyset with key_index for
# config 5).
@pytest.mark.parametrize("config,records", [("config2", 4096), ("config4", 8192)])
def test_bench_layout_reference_digest(config, records):
    w = bench.build_workload(config, 0, 1, records, torch.device("cuda:0"), open_op=True)
    assert bool(w.d_status[:w.nrec].all())
    code, parity = bench.verify_workload(w)
    assert code == bench.PARITY_OK, parity
    w.d_status.zero_()
    w.op(w.batch, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert bool(w.d_status[:w.nrec].all()) and torch.equal(w.d_back, w.d_pt)


@pytest.mark.parametrize("config,records", [("configG", 6000), ("config5", 64 * 40)])
def test_bench_layout_vs_oracle(config, records):
    aead, key_len = bench.CONFIGS[config][0], bench.CONFIGS[config][1]
    w = bench.build_workload(config, 0, 1, records, torch.device("cuda:0"))
    w.op(w.batch, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert bool(w.d_status[:w.nrec].all())
    n, lens = w.nrec, w.lens
    pt, offs, nonces, ads = o.synth_batch(0, lens, align=bench.record_align(config))
    rpk = bench.RECORDS_PER_KEY.get(config)
    if rpk:
        nk = (n + rpk - 1) // rpk
        keys = o.synth_keys(nk, key_len)
        kidx = (np.arange(n) // rpk).astype(np.uint32)
    else:
        keys = np.frombuffer(o.synth_key(0, key_len), dtype=np.uint8).copy()
        kidx = None
    out = np.zeros_like(pt)
    tags = np.zeros(16 * n, dtype=np.uint8)
    assert o.batch(o.AES_GCM, 1, keys, key_len, kidx, pt, out, offs, lens, nonces, 12, ads,
                   np.arange(n, dtype=np.uint64) * np.uint64(13), np.full(n, 13, np.uint64),
                   tags, 16) == 0
    got = w.d_ct[:pt.size].cpu().numpy()
    assert np.array_equal(got, out)
    assert np.array_equal(w.d_tags[:16 * n].cpu().numpy(), tags)


# The record end's own E_K(J0) (gcm_bs.hip self_ek0): with
# the batched production switched off (include/bssl_amd/test_hooks.h), every
# record end waits its bounded number of polls for granules that never come,
# then computes its E_K(J0) itself -- one-key (uniform and ragged, both
# lane counts), keyset and non-96-bit-nonce batches, seal and open.
@pytest.fixture
def no_ek0_producers():
    prev = ba.test_set_bs_ek0_producers(False)
    yield
    ba.test_set_bs_ek0_producers(prev)


@pytest.mark.parametrize("aead", GCM)
def test_ek0_fallback_ragged_vs_oracle(aead, no_ek0_producers):
    par.test_batch_ragged_vs_oracle(aead, "aligned")


@pytest.mark.parametrize("multikey", [False, True])
def test_ek0_fallback_large_ragged(multikey, no_ek0_producers):
    par.test_batch_large_ragged_reordered("aes-128-gcm", multikey)


def test_ek0_fallback_nonce_lengths(no_ek0_producers):
    par.test_batch_gcm_nonce_lengths_and_truncated_tags()


def test_ek0_fallback_bench_layout(no_ek0_producers):
    test_bench_layout_reference_digest("config2", 4096)
