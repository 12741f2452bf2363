set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/ab_anyal/libbssl_amd.so
timeout -k 10 1200 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
for al in 128 16; do
  BSSL_AMD_ALIGN=$al timeout -k 10 300 python bench.py --config config3 --no-cpu-baseline > gpurun_out/b_config3_a$al.log 2>&1 || exit 1
  echo "anyal config3 align=$al $(grep -o '"value": [0-9.]*\|"parity": "[^"]*"' gpurun_out/b_config3_a$al.log | tr '\n' ' ')"
done
timeout -k 10 300 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 2>&1 | grep "^{"
unset BSSL_AMD_LIB
timeout -k 10 300 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 2>&1 | grep "^{"
