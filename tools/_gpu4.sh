cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
for lf in 0 1; do SDFNMPC_LIN_FIRST=$lf timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 2> gpurun_out/b.err | python3 -c "import json,sys; d=json.load(sys.stdin); print('lin_first=$lf', round(d['value']), round(d['ms_per_step']*1e3,1), 'us', {k:round(v*1e3,1) for k,v in d['kernel_ms'].items()}, round(d['roofline']['achieved'],1))" || { tail gpurun_out/b.err; exit 3; }; done
