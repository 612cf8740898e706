#!/bin/bash
# Experiment: every kernel built with LLVM's max-ilp AMDGPU scheduling strategy (_build/maxilp) against the
# product library: preparation phase, wide-net preparation, VAE encode; the QP through its drivers
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
O=$R/gpurun_out/maxilp; mkdir -p $O; : > $O/out.txt
for lib in product maxilp; do
  L=$R/sdf-nmpc_amd/lib/libsdfnmpc.so; [ $lib = maxilp ] && L=$R/_build/maxilp/libsdfnmpc.so
  echo "== $lib" >> $O/out.txt
  SDFNMPC_LIB=$L timeout -k 10 120 python3 tools/sdf_bench.py 2>&1 | grep ms/prep >> $O/out.txt
  SDFNMPC_LIB=$L timeout -k 10 120 python3 tools/wide_bench.py 2>&1 | grep -E "ms/prep|gemm" >> $O/out.txt
  SDFNMPC_LIB=$L timeout -k 10 120 python3 tools/vae_bench.py 2>&1 | grep -E "ms/encode|stem|conv" >> $O/out.txt
done
for d in _vf _max-ilp _vf _max-ilp; do echo "qp $d: $(DRV=$d B=1024 N=40 timeout -k 10 120 python3 tools/qp_stamps.py 2>&1 | grep kernel)" >> $O/out.txt; done
cat $O/out.txt
