# late round-4 profiles: rocprofv3 trace + PMC passes of the workloads whose kernels changed
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
source "$R/tools/configs.sh"
for t in "$@"; do
  bash "$R/tools/profile_config.sh" "r04l/$t" ${CFG[$t]} || exit $?
done
echo "profiles ok"
