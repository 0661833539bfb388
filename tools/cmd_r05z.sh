# r05z: static wave priority in the row kernel (none / waves 4-7 / waves 0-3 at s_setprio 1);
# kernel trace of the headline (overlapped, unprofiled) bench pass for tools/busy.py;
# SQ counters of k_item_attn
export NPFN_AB_KERNELS=1 TMPDIR=/tmp
mkdir -p gpurun_out/r05z
timeout -k 10 1100 python -u tools/ab_bench.py 4 tools/diaglib/libnpfn_prio0.so tools/diaglib/libnpfn_prio1.so tools/diaglib/libnpfn_prio2.so > gpurun_out/r05z/ab.txt 2>&1; tail -7 gpurun_out/r05z/ab.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05z/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --prof-steps 0 > gpurun_out/r05z/kt.json 2> gpurun_out/r05z/kt.err && \
python tools/busy.py gpurun_out/r05z/kt/kt_kernel_trace.csv k_fill 6 > gpurun_out/r05z/busy.txt; tail -25 gpurun_out/r05z/busy.txt
bash tools/gpu_sq.sh r05z_ia k_item_attn
