# round-end set on the final tree: whole GPU suite, smoke(), the default bench line
#   bash tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
trc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -8
[ $trc -eq 0 ] || [ $trc -eq 1 ] || exit $trc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])
print('kitti', d['secondary']['images_per_sec'])
for k,v in d['secondaries'].items(): print(k, v.get('images_per_sec', v.get('gpu_images_per_sec')), v.get('ms_per_step'), (v.get('roofline') or {}).get('bound'), (v.get('roofline') or {}).get('frac'))"
exit $trc
