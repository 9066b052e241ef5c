set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_knob_ab.py --variants 'igemm:halo=0;halo:halo=1;noDMA:halo_dbg=1;noEPI:halo_dbg=2;noMFMA:halo_dbg=4;MFMAonly:halo_dbg=3;DMAonly:halo_dbg=6' --only l1_3x3 --modes fwd,dgrad > gpurun_out/halo_dbg.log 2>&1 || { tail -20 gpurun_out/halo_dbg.log; exit 1; }
grep -v amdgpu gpurun_out/halo_dbg.log
