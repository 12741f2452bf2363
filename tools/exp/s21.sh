set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/boringssl_amd/csrc/build
BSSL_AMD_LIB=$B/ab_stamps/libbssl_amd.so timeout -k 10 300 python bench.py --config configG --steps 1 --warmup 0 --no-cpu-baseline --no-parity > gpurun_out/s21_stamps_G.txt 2>&1 || exit 1
BSSL_AMD_LIB=$B/ab_stamps/libbssl_amd.so timeout -k 10 300 python bench.py --config config2 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > gpurun_out/s21_stamps_2.txt 2>&1 || exit 1
grep -h "stamps block 0" gpurun_out/s21_stamps_G.txt | head -16
grep -h "stamps block 0" gpurun_out/s21_stamps_2.txt | head -4
SPECS="configG:ab_nofin config4:ab_nofin" REPS="1 2" timeout -k 10 600 bash tools/exp/ab_session.sh > gpurun_out/s21_ab.txt 2>&1; cat gpurun_out/s21_ab.txt
timeout -k 10 300 python bench.py --config configG > gpurun_out/s21_G.json 2>gpurun_out/s21_G.err; tail -1 gpurun_out/s21_G.json
