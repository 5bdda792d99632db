#!/bin/bash
# GPU box: calibration + the roofline profiles of the BASELINE configs (and model_4).
#   tools/gpu_profiles.sh <round> [tag ...]   (default: every tag below)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
RND=$1
shift
declare -A CFG=(
  [glide]=""                                               # BASELINE config 2
  [s3]="--ne 250 --nc 114"                                 # config 3 shapes
  [s5]="--ne 250 --nc 150"                                 # config 4, per GPU
  [stress]="--ne 1024 --nc 512 --batch 32"                 # config 5, per GPU
  [m4_glide]="--variant 4"                                 # full HD-GNN
  [m4_stress]="--variant 4 --ne 1024 --nc 512 --batch 32"
)
TAGS=${*:-"glide s3 s5 stress m4_glide m4_stress"}
if [ ! -f "$R/gpurun_out/$RND/cal/done" ]; then
  bash "$R/tools/calibrate.sh" "$RND" || exit $?
  touch "$R/gpurun_out/$RND/cal/done"
fi
for t in $TAGS; do
  bash "$R/tools/profile_config.sh" "$RND/$t" ${CFG[$t]} || exit $?
done
echo "profiles ok"
