#!/bin/bash
# round 4: persistent hubfactor grid on the 20ng shape; rocminfo CU count
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('CUs', p.multi_processor_count, p.name)"
for v in product p128 p240; do
  lib=""; [ $v != product ] && lib="GCNK_LIB=$PWD/_variants/libgcnk_$v.so"
  env $lib timeout -k 10 200 python -u scripts/factor_probe.py --graphs 20ng > gpurun_out/r04/fp20_$v.log 2>&1; echo "$v rc=$?"
  grep "hubfactor\|forward" gpurun_out/r04/fp20_$v.log
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/fp20_prof -o fp -- python3 scripts/factor_probe.py --graphs 20ng > gpurun_out/r04/fp20_prof.log 2>&1; echo "prof rc=$?"
grep -h "hubfactor" gpurun_out/r04/fp20_prof/*kernel_stats.csv | cut -d, -f1-8 | cut -c1-220
