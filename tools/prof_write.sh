# WRITE_SIZE pass restricted to the GEMM kernels (+ adamw, the step marker):
# an unrestricted WRITE_SIZE pass segfaults inside the profiler on this image.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'gemm_f32_kernel|adamw_kernel' -d gpurun_out/r01_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r01_write.log 2>&1
