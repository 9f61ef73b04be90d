cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_ab
mkdir -p $O
cd $R/abtree && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/old -o run -- python3 $R/abtree/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/old.log 2>&1 || exit 1
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/new -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/new.log 2>&1 || exit 1
ls $O/old $O/new
