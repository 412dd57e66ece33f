# rocprofv3 exit-time SIGSEGV hunt: the bench without the cooperative accumulation launch
# (MC_ACCUM_STEPS=1: host-driven get_close steps), small config
R=$GRAFT_REPO_ROOT; cd $R && export TMPDIR=/tmp
MC_ACCUM_STEPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pe3 -o run -- python3 bench.py --n 20000 --templates 200 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pe3.log 2>&1; echo rc=$? >> $R/gpurun_out/pe3.log
