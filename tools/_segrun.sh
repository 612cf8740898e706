# diagnostic: per-phase stamps of the segmented QP kernel at P = 2, 3, 4 (B = 1024 and B = 64), then timing
mkdir -p gpurun_out
for P in 2 3 4; do
  SDFNMPC_QP_NSEG=$P DRV=_seg timeout -k 10 100 python -u tools/qp_stamps.py > gpurun_out/seg_stamps_P$P.log 2>&1 || exit 1
  B=64 SDFNMPC_QP_NSEG=$P DRV=_seg timeout -k 10 100 python -u tools/qp_stamps.py > gpurun_out/seg_stamps_P${P}_b64.log 2>&1 || exit 1
done
SDFNMPC_QP_NSEG=3 timeout -k 10 200 python -u tools/seg_check.py 8,40,2 1024,40,5 > gpurun_out/seg_check.log 2>&1 || exit 1
for P in 2 4; do SDFNMPC_QP_NSEG=$P timeout -k 10 200 python -u tools/seg_check.py 1024,40,5 > gpurun_out/seg_check_P$P.log 2>&1 || exit 1; done
