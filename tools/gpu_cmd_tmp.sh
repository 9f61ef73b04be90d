cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "probes" > gpurun_out/t_p.txt 2>&1 || { tail -30 gpurun_out/t_p.txt; exit 1; }
tail -2 gpurun_out/t_p.txt
timeout -k 10 120 python -u -c "
import sd_amd_loader; sd_amd_loader.load()
from sd_amd import ops
for i in range(3): print(ops.probe_peaks())
" 2>&1 | grep -v amdgpu.ids
