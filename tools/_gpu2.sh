cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { tail gpurun_out/bench2.err; exit 3; }
cat gpurun_out/bench2.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc1 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1 || { tail -20 gpurun_out/pmc1.log; exit 4; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1 || { tail -20 gpurun_out/pmc2.log; exit 5; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc3.log 2>&1 || { tail -20 gpurun_out/pmc3.log; echo pmc3 failed; }
ls gpurun_out/pmc1 gpurun_out/pmc3
