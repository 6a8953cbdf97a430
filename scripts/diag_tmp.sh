set -e
mkdir -p gpurun_out/diag1
SG_LIB=graphembedding_amd/lib/libsiamese_timing.so timeout -k 10 120 python scripts/fast_timing.py 1 8 > gpurun_out/diag1/timing.log 2>&1
timeout -k 10 120 python bench.py --emulate-world 8 --steps 200 --warmup 20 --cpu-sample -1 > gpurun_out/diag1/emu8.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/diag1/trace8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --emulate-world 8 --steps 50 --warmup 5 --cpu-sample -1 > $GRAFT_REPO_ROOT/gpurun_out/diag1/trace8.log 2>&1
