set -u
L=graphembedding_amd/lib
SKIP_TESTS= bash scripts/gpu_c5_var.sh r3c_c5 rows8= rows4=SG_LIB=$L/libsiamese_c5a.so,SG_WEB_XCD=0 || exit $?
TESTS="tests/test_gpu_parity.py tests/test_gpu_fullbatch.py tests/test_gpu_order.py" TEST_ENV="SG_LIB=$L/libsiamese_nie.so" \
  bash scripts/gpu_var.sh r3c_c2 base= nie=SG_LIB=$L/libsiamese_nie.so || exit $?
TESTS="tests/test_gpu_fast32.py" TEST_ENV="SG_LIB=$L/libsiamese_nie32.so" BENCH_ARGS="--dataset syn_aids10knef --steps 3 --warmup 1" \
  bash scripts/gpu_var.sh r3c_c4 base= nie32=SG_LIB=$L/libsiamese_nie32.so ilp=SG_LIB=$L/libsiamese_c4ilp.so p12=SG_LIB=$L/libsiamese_c4p12.so || exit $?
