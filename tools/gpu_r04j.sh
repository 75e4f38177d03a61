# round 4: critical path of the contacts-on quad and obstacle rollout kernels (stamped build, last
# step of 20-step launches), PMC passes of the obstacle rollout kernel, then a bench line with the
# secondary / obstacle legs' roofline blocks
set -o pipefail
mkdir -p gpurun_out
cp profiles/critical_path_latest.json gpurun_out/critical_path.json
STAMPS_ROLLOUT=20 STAMPS_JSON=gpurun_out/critical_path.json timeout -k 10 200 python -u tools/stamps.py quad > gpurun_out/r04j_stamps_quad.log 2>&1 || { echo STAMPS_Q_FAIL; tail -20 gpurun_out/r04j_stamps_quad.log; exit 1; }
STAMPS_ROLLOUT=20 STAMPS_JSON=gpurun_out/critical_path.json timeout -k 10 200 python -u tools/stamps.py obst > gpurun_out/r04j_stamps_obst.log 2>&1 || { echo STAMPS_O_FAIL; tail -20 gpurun_out/r04j_stamps_obst.log; exit 1; }
grep -A9 "^==" gpurun_out/r04j_stamps_quad.log gpurun_out/r04j_stamps_obst.log
timeout -k 10 300 python3 tools/profile_pmc.py 20,1000 --obstacles > gpurun_out/r04j_pmc_obst.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/r04j_pmc_obst.log; exit 1; }
grep -o '"hbm_bytes_per_step": [0-9.]*\|"valu_insts_per_wave_step": [0-9.]*' gpurun_out/r04j_pmc_obst.log
