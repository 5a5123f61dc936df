# round-6 final tree: whole GPU suite, smoke(), default bench line, then bench --ddp (world-1 group + overlap model)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_final.sh r6k || exit $?
timeout -k 10 600 python -u bench.py --ddp --no-cpu-baseline --no-secondary > gpurun_out/r6k_ddp.json 2> gpurun_out/r6k_ddp.err || { tail -20 gpurun_out/r6k_ddp.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r6k_ddp.json').read().strip().splitlines()[-1])
print(d['value'], json.dumps(d.get('allreduce'))[:1500])"
