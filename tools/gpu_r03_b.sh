#!/bin/bash
# round-3 check: NAS train + new parity tests, A/Bs of the new kernels, NAS train bench, NAS / c5 PMC
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nas_train.py tests/test_gpu_parity.py -s -v --timeout 120 --timeout-method thread -k "nas_train or supernet or front or two_block or candidate" > gpurun_out/r03b_pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/r03b_pytest.log | tail -2
ENVS="-;HN_PAIRDIST_REG=1" REPS=2 BENCH_ARGS="--config 5 --steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
ENVS="-;HN_NO_IRF2=1;HN_FRONT_FOLD=1" REPS=2 BENCH_ARGS="--model wang2 --steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
ENVS="-;HN_NO_IRF2=1" REPS=1 BENCH_ARGS="--model wang4 --steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
timeout -k 10 300 python tools/bench_train_nas.py > gpurun_out/bench_train_nas.json 2> gpurun_out/bench_train_nas.err || { tail -5 gpurun_out/bench_train_nas.err; exit 1; }
cat gpurun_out/bench_train_nas.json
timeout -k 10 200 python tools/bench_train.py > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err || { tail -5 gpurun_out/bench_train.err; exit 1; }
cat gpurun_out/bench_train.json
MODELS="wang2 wang3 wang4 c5" timeout -k 10 900 bash tools/pmc_all.sh > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
echo pmc done
