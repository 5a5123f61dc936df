# ODA2 ordered-swin2: bench line with the CPU baseline, then kernel trace + GEMM PMC traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --model oda2 --steps 5 --warmup 2 > gpurun_out/r4w_oda2.json 2> gpurun_out/r4w_oda2.err || { tail -20 gpurun_out/r4w_oda2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4w_oda2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d.get('cpu_baseline'))"
bash tools/prof_round.sh r4_oda2 --model oda2 || exit 1
echo oda2 prof done
