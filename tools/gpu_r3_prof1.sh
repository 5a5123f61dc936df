# round 3: ODA2 bench line; PMC traffic for the KITTI secondary (fp32 GEMMs) and the bf16 GEMM family
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --model oda2 --steps 3 --warmup 2 --cpu-budget-s 20 > gpurun_out/bench_oda2.log 2>&1 || { tail -20 gpurun_out/bench_oda2.log; exit 1; }
grep '^{"metric' gpurun_out/bench_oda2.log | cut -c1-400
bash tools/prof_traffic.sh r3k 'gemm_f32_kernel' --model newcrfs_kitti
bash tools/prof_traffic.sh r3bf 'gemm_m16_kernel' --model depthformer --precision bf16
