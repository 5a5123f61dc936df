# round-6 refresh of the two lines the default bench does not carry: ODA2 ordered-swin2 and the file front end
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --model oda2 --steps 3 --warmup 2 > gpurun_out/r6v_oda2.json 2> gpurun_out/r6v_oda2.err || { tail -20 gpurun_out/r6v_oda2.err; exit 1; }
tail -c 400 gpurun_out/r6v_oda2.json
timeout -k 10 600 python -u bench.py --data synthetic-files --no-cpu-baseline --no-secondary > gpurun_out/r6v_files.json 2> gpurun_out/r6v_files.err || { tail -20 gpurun_out/r6v_files.err; exit 1; }
tail -c 400 gpurun_out/r6v_files.json
