"""The experimental mixed-role AES-GCM engine (gcm_mix.hip, round 6, VERDICT
r5 item 2): NB of each workgroup's 16 waves run the table-free engine
(bitsliced AES, gcm_bs.hip bs_unit), the others the T-table engine (gcm.hip
process_records), on one unit counter.  Every record and tag against the CPU
oracle (oracle/aead_oracle.c, following gcm.cc.inc:298-604) for NB = 2, 4, 6;
open in place with a tampered record; the bench's config-2 layout at reduced
size against the reference library's digest.
"""
import os
import sys
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import boringssl_amd as ba  # noqa: E402
import oracle_lib as o  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(params=[2, 4, 6])
def mix(request):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    prev = ba.test_set_gcm_mix(request.param)
    yield request.param
    ba.set_aes_gcm_engine(prev)


@pytest.mark.parametrize("rlen,n", [(4096, 1000), (16384, 333), (8208, 257)])
def test_mix_uniform_vs_oracle(mix, rlen, n):
    rng = np.random.default_rng(zlib.crc32(repr((mix, rlen, n)).encode()))
    key = rng.integers(0, 256, size=16, dtype=np.uint8).tobytes()
    recs = rng.integers(0, 256, size=(n, rlen), dtype=np.uint8)
    nonces = rng.integers(0, 256, size=n * 12, dtype=np.uint8)
    ad = rng.integers(0, 256, size=n * 13, dtype=np.uint8)
    d_pt = torch.from_numpy(recs.reshape(-1).copy()).to(DEV)
    d_ct = torch.zeros_like(d_pt)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=DEV)
    d_st = torch.zeros(n, dtype=torch.uint8, device=DEV)
    d_n = torch.from_numpy(nonces).to(DEV)
    d_ad = torch.from_numpy(ad).to(DEV)
    ctx = ba.AEADCtx("aes-128-gcm", key, 16)
    b = ba.make_batch(n, d_pt, d_ct, d_tags, d_n, 12, d_ad, record_stride=rlen, record_len=rlen,
                      ad_stride=13, ad_len=13, status=d_st)
    ba.set_kernel_timing(True)
    ctx.seal_batch_device(b)
    torch.cuda.synchronize()
    ba.collect_kernel_times()
    ba.set_kernel_timing(False)
    assert ba.last_kernel_name() == "gcm_mix_kernel"
    assert bool(d_st.all())
    flat = recs.reshape(-1)
    ref = np.zeros_like(flat)
    ref_tags = np.zeros(16 * n, dtype=np.uint8)
    assert o.batch(o.AES_GCM, 1, np.frombuffer(key, dtype=np.uint8).copy(), 16, None, flat, ref,
                   np.arange(n, dtype=np.uint64) * np.uint64(rlen), np.full(n, rlen, np.uint64),
                   nonces, 12, ad, np.arange(n, dtype=np.uint64) * np.uint64(13),
                   np.full(n, 13, np.uint64), ref_tags, 16) == 0
    got = d_ct.cpu().numpy().reshape(n, rlen)
    bad = np.nonzero((got != ref.reshape(n, rlen)).any(axis=1))[0]
    assert bad.size == 0, f"records differ from the oracle: {bad[:8].tolist()}"
    assert np.array_equal(d_tags.cpu().numpy(), ref_tags)
    # open in place, one tampered record
    ct = d_ct.clone()
    ct[7 * rlen + 100] ^= 4
    d_st.zero_()
    b2 = ba.make_batch(n, ct, ct, d_tags, d_n, 12, d_ad, record_stride=rlen, record_len=rlen,
                       ad_stride=13, ad_len=13, status=d_st)
    ctx.open_batch_device(b2)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    assert [i for i in range(n) if not st[i]] == [7]
    back = ct.cpu().numpy().reshape(n, rlen)
    assert not back[7].any()
    keep = np.ones(n, dtype=bool)
    keep[7] = False
    assert np.array_equal(back[keep], recs[keep])


def test_mix_bench_layout_reference_digest(mix):
    w = bench.build_workload("config2", 0, 1, 4096, torch.device(DEV))
    w.op(w.batch, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert bool(w.d_status[:w.nrec].all())
    code, parity = bench.verify_workload(w)
    assert code == bench.PARITY_OK, parity
