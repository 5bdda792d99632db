# GPU box: prepare-kernel timings of ablation builds (HDG_LIB_PATH), kernel traces only.
set -o pipefail
R=${GRAFT_REPO_ROOT}
mkdir -p $R/gpurun_out/prepabl
cd /tmp && export TMPDIR=/tmp
for v in "" _abl1 _abl2; do
  HDG_LIB_PATH=$R/hd-gnn_amd/csrc/libhdgnn$v.so timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/prepabl/t$v -o run -- python3 $R/tools/prep_time.py > $R/gpurun_out/prepabl/t$v.log 2>&1 || exit $?
  echo "done $v"
done
