# diagnostic: per-phase stamps of the segmented QP kernel (B = 1024 and B = 64)
mkdir -p gpurun_out
P=${P:-3}
SDFNMPC_QP_NSEG=$P DRV=_seg timeout -k 10 100 python -u tools/qp_stamps.py > gpurun_out/seg_stamps.log 2>&1 || exit 1
B=64 SDFNMPC_QP_NSEG=$P DRV=_seg timeout -k 10 100 python -u tools/qp_stamps.py > gpurun_out/seg_stamps_b64.log 2>&1 || exit 1
