export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 200 ./tools/microbench 1048576 200 copy > gpurun_out/mb_copy.log 2>&1 && cat gpurun_out/mb_copy.log &&
timeout -k 10 300 python bench.py --config nat64_4to6 --steps 300 --warmup 30 --cpu-seconds 5 > gpurun_out/bench_4to6.log 2>&1 && tail -1 gpurun_out/bench_4to6.log &&
timeout -k 10 300 python bench.py --config nat64_4to6 --e2e --steps 300 --warmup 30 > gpurun_out/e2e_4to6.log 2>&1 && tail -1 gpurun_out/e2e_4to6.log
