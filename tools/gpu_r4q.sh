# round-4 PMC traffic of the other workloads: Depthformer fp32, Depthformer bf16 (eager: PMC passes
# over graph replays hung), AdaBins; kernel trace + FETCH_SIZE + WRITE_SIZE each
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_round.sh r4_df32 --model depthformer --no-secondary || exit 1
echo df32 done
KREGEX='gemm_m16_kernel|adamw' bash tools/prof_round.sh r4_dfb --model depthformer --precision bf16 --no-secondary || exit 1
echo dfb done
bash tools/prof_round.sh r4_ada --model adabins --no-secondary || exit 1
echo ada done
