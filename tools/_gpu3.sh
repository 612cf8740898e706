cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x -k "sdf" > gpurun_out/pytest_sdf.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_sdf.log; [ $rc -gt 1 ] && exit $rc
for t in 32 64; do timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --tile-rows $t 2> gpurun_out/b.err | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['kernel_ms'], d['roofline']['achieved'])" || { tail gpurun_out/b.err; exit 3; }; done
