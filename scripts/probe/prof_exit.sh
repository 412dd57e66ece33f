# rocprofv3 on the libmcgpu probe, without and with torch (exit-time SIGSEGV hunt)
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pe1 -o run -- python3 $R/scripts/probe/prof_exit.py $R/gpurun_out/pe1_maps.txt > $R/gpurun_out/pe1.log 2>&1; echo rc=$? >> $R/gpurun_out/pe1.log
