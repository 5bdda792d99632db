# tag -> bench.py arguments of every workload the round's evidence covers (BASELINE configs x
# model variants x engine paths); sourced by tools/gpu_profiles.sh and tools/bench_matrix.sh
declare -A CFG=(
  [glide]=""                                               # BASELINE config 2 (model_2, fused)
  [m2_general_glide]="--path 2"
  [m1_glide]="--variant 1"
  [m3_glide]="--variant 3"
  [m4_glide]="--variant 4"                                 # full HD-GNN (hybrid)
  [m4_general_glide]="--variant 4 --path 2"
  [s3]="--ne 250 --nc 114"                                 # config 3 shapes
  [s5]="--ne 250 --nc 150"                                 # config 4, per GPU
  [m4_s5]="--variant 4 --ne 250 --nc 150"
  [m4_general_s5]="--variant 4 --ne 250 --nc 150 --path 2"
  [stress]="--ne 1024 --nc 512 --batch 32"                 # config 5, per GPU
  [m4_stress]="--variant 4 --ne 1024 --nc 512 --batch 32"
)
ORDER="glide m2_general_glide m1_glide m3_glide m4_glide m4_general_glide s3 s5 m4_s5 m4_general_s5 stress m4_stress"
