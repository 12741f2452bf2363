set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "chacha or uniform or baseline_config_digest or iov or Sealv or Openv" --timeout 300 --timeout-method thread > gpurun_out/t_main.log 2>&1 || { tail -20 gpurun_out/t_main.log; exit 1; }
tail -1 gpurun_out/t_main.log
BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/ab_pers4/libbssl_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "chacha or uniform or baseline_config_digest" --timeout 300 --timeout-method thread > gpurun_out/t_pers4.log 2>&1 || { tail -20 gpurun_out/t_pers4.log; exit 1; }
tail -1 gpurun_out/t_pers4.log
SPECS="config3:ab_pers4,ab_pers8 config3x:ab_pers4,ab_pers8,ab_x4" REPS="1 2" timeout -k 10 900 bash tools/exp/ab_session.sh > gpurun_out/ab_pers.txt 2>&1; cat gpurun_out/ab_pers.txt
timeout -k 10 300 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 2>&1 | grep '^{'
BSSL_AMD_LIB=$PWD/boringssl_amd/csrc/build/ab_iovl4/libbssl_amd.so timeout -k 10 300 python tools/iov_bench.py --aead chacha20-poly1305 --records 1048576 --len 1350 2>&1 | grep '^{'
timeout -k 10 300 python tools/iov_bench.py --aead xchacha20-poly1305 --records 1048576 --len 1350 2>&1 | grep '^{'
