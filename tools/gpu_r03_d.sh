#!/bin/bash
# round-3 check: k_head3 (split rings) and the NAS fused uint8 front; head A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_preprocess.py -m gpu -v --timeout 120 --timeout-method thread -k "head_forms or reference_vectors or timed_size or forward_u8" > gpurun_out/r03d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r03d_pytest.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r03d_pytest.log | head; exit 1; }
ENVS="-;HN_HEAD=4;HN_HEAD=2" REPS=2 BENCH_ARGS="--steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
ENVS="-;HN_HEAD=2" REPS=1 BENCH_ARGS="--model wang2 --steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
ENVS="-" REPS=1 BENCH_ARGS="--model wang2 --input u8-cv2 --steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
