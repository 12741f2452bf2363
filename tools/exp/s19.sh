set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=boringssl_amd/csrc/build/ab_iovd/libbssl_amd.so
BSSL_AMD_LIB=$PWD/$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k iovec > gpurun_out/s19_tests.txt 2>&1 || { tail -30 gpurun_out/s19_tests.txt; exit 1; }
tail -2 gpurun_out/s19_tests.txt
for rep in 1 2; do
  for a in chacha20-poly1305 xchacha20-poly1305; do
    for len in 1350 16384; do
      n=$(( len == 1350 ? 1048576 : 131072 ))
      echo "== $rep $a $len main"; timeout -k 10 120 python tools/iov_bench.py --aead $a --records $n --len $len || exit 1
      echo "== $rep $a $len iovd"; BSSL_AMD_LIB=$PWD/$V timeout -k 10 120 python tools/iov_bench.py --aead $a --records $n --len $len || exit 1
    done
  done
done 2>&1 | tee gpurun_out/s19.txt
