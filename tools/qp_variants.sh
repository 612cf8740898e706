# build QP timing-driver variants (diagnostic): tools/qp_variants.sh NAME "EXTRA FLAGS" ...
cd "$(dirname "$0")/.."
while [ $# -gt 1 ]; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -I sdf-nmpc_amd/csrc $2 tools/qp_stamps_drv.hip sdf-nmpc_amd/csrc/rti_qp.hip -o tools/_qp_stamps_drv_$1 2>&1 | grep error
  shift 2
done
