# rocprofv3 on a small bench run with the process map dumped (exit-time SIGSEGV hunt)
R=$GRAFT_REPO_ROOT; cd $R && export TMPDIR=/tmp
MC_DUMP_MAPS=$R/gpurun_out/pe2_maps.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pe2 -o run -- python3 bench.py --n 20000 --templates 200 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pe2.log 2>&1; echo rc=$? >> $R/gpurun_out/pe2.log
