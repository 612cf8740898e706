set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
for cfg in "5 0.05" "17 0.3" "29 1.0"; do
  set -- $cfg
  SEED=$1 NOISE=$2 timeout -k 10 200 python $R/tools/qp_stamps.py > /dev/null 2>&1 || true
  echo "#### seed $1 x0 noise $2"
  for d in $R/tools/_qp_stamps_drv_*; do echo -n "$(basename $d): "; timeout -k 10 60 $d /tmp/qp_in.bin | head -1; done
done
