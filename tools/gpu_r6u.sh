# the default bench line on the final tree (event timing behind spin kernels), then bench --ddp (bucket rebuild)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r6u_bench.json 2> gpurun_out/r6u_bench.err || { tail -20 gpurun_out/r6u_bench.err; exit 1; }
tail -c 300 gpurun_out/r6u_bench.json
timeout -k 10 300 python -u bench.py --ddp --no-cpu-baseline --no-secondary > gpurun_out/r6u_ddp.json 2> gpurun_out/r6u_ddp.err || { tail -20 gpurun_out/r6u_ddp.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r6u_ddp.json').read().strip().splitlines()[-1])
ov=d['allreduce']['overlap']; print(d['value'], d['allreduce']['buckets'], ov['ready_order'], ov['ready_order_is_index_order'], ov['held_back_buckets'], ov['model_exposed_ms'])"
