set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_block_gpu.py tests/test_fp8_stem_gpu.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c1_tests.log 2>&1; rc=$?; tail -3 gpurun_out/c1_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 > gpurun_out/c1_infer_block.log 2>&1 || exit $?
grep '"value"\|speedup' gpurun_out/c1_infer_block.log
FN_F8_BLOCK=0 timeout -k 10 300 python bench/infer_fp8.py --size 128 --batch 1024 --chunk 1024 --only fp8 > gpurun_out/c1_infer_tensor.log 2>&1 || exit $?
grep '"value"' gpurun_out/c1_infer_tensor.log
timeout -k 10 300 python scripts/bench_fc_native.py --batch 128 --reps 50 > gpurun_out/c1_fc.log 2>&1 || exit $?
tail -1 gpurun_out/c1_fc.log
timeout -k 10 400 python -u -m pytest tests/test_determinism_gpu.py tests/test_bnfuse_gpu.py tests/test_gpu_pipeline.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c1_det.log 2>&1; rc=$?; tail -3 gpurun_out/c1_det.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/c1_bench.log 2>&1 || exit $?
tail -1 gpurun_out/c1_bench.log | cut -c1-300
timeout -k 10 300 python scripts/diag_step_kernels.py --small-us 20 > gpurun_out/c1_diag.log 2>&1 || exit $?
tail -3 gpurun_out/c1_diag.log
timeout -k 10 300 python scripts/diag_nas_step.py --list > gpurun_out/c1_nas.log 2>&1 || exit $?
tail -1 gpurun_out/c1_nas.log
