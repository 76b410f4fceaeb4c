# BC (backward adjoint) channel-group sweep on the trainer sizes: GNCA_BC_WGS_PER_CU = 2, 4, 8, 16.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for n in 2 4 8 16; do
  GNCA_BC_WGS_PER_CU=$n timeout -k 10 200 python tools/time_bwd.py --sizes 16x128 --channels 32 --radius 5 --k 16 --iters 10 2>/dev/null | sed "s/^/wgs_per_cu=$n /" | grep fwd
  GNCA_BC_WGS_PER_CU=$n timeout -k 10 200 python tools/time_bwd.py --sizes 16x40 --iters 20 2>/dev/null | sed "s/^/wgs_per_cu=$n /" | grep fwd
done
