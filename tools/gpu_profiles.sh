#!/bin/bash
# GPU box: calibration + the roofline profiles of every workload in tools/configs.sh.
#   tools/gpu_profiles.sh <round> [tag ...]   (default: all, in ORDER)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
source "$R/tools/configs.sh"
RND=$1
shift
TAGS=${*:-$ORDER}
# NOCAL=1: skip the counter calibration (profiles/<round>/calibration.json already committed)
if [ -z "$NOCAL" ] && [ ! -f "$R/gpurun_out/$RND/cal/done" ]; then
  bash "$R/tools/calibrate.sh" "$RND" || exit $?
  touch "$R/gpurun_out/$RND/cal/done"
fi
for t in $TAGS; do
  bash "$R/tools/profile_config.sh" "$RND/$t" ${CFG[$t]} || exit $?
done
echo "profiles ok"
