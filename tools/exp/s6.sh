set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "iov or Sealv or Openv" --timeout 300 --timeout-method thread > gpurun_out/iov_tests.log 2>&1 || { tail -30 gpurun_out/iov_tests.log; exit 1; }
tail -1 gpurun_out/iov_tests.log
for a in "aes-128-gcm" "aes-128-gcm --in-gap 0 --out-gap 0" "chacha20-poly1305 --records 1048576 --len 1350" "xchacha20-poly1305 --records 1048576 --len 1350" "aes-128-gcm-siv"; do
timeout -k 10 300 python tools/iov_bench.py --aead $a 2>&1 | grep '^{' || exit 1
done
