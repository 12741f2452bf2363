set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "iovec" --timeout 300 --timeout-method thread > gpurun_out/iov_tests.log 2>&1 || { tail -30 gpurun_out/iov_tests.log; exit 1; }
tail -2 gpurun_out/iov_tests.log
for a in chacha20-poly1305 xchacha20-poly1305; do
timeout -k 10 300 python tools/iov_bench.py --aead $a --records 1048576 --len 1350 > gpurun_out/iov_$a.json 2>&1 || exit 1
cat gpurun_out/iov_$a.json
done
timeout -k 10 300 python tools/iov_bench.py --aead aes-128-gcm > gpurun_out/iov_gcm.json 2>&1 && cat gpurun_out/iov_gcm.json
STEPS="smoke pytest bench" bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python bench.py --config config3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit 1
timeout -k 10 300 python tools/e2e_bench.py --config config3 --chunk 65536 > gpurun_out/e2e_c3.log 2>&1
cat gpurun_out/e2e_c3.log
timeout -k 10 300 python tools/iov_bench.py --aead aes-128-gcm-siv > gpurun_out/iov_siv.json 2>&1 && cat gpurun_out/iov_siv.json
timeout -k 10 300 python tools/iov_bench.py --aead aes-128-gcm --in-gap 0 --out-gap 0 > gpurun_out/iov_gcm00.json 2>&1 && cat gpurun_out/iov_gcm00.json
SPECS="config3:sdwa,unr5,unr2,ntl,prio0,l2,l2t512" timeout -k 10 900 bash tools/exp/ab_session.sh > gpurun_out/ab.txt 2>&1; cat gpurun_out/ab.txt
