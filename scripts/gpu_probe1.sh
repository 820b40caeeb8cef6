export TMPDIR=/tmp
O=gpurun_out/probe1; mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1; echo list=$?
timeout -k 10 300 python -u scripts/lane_probe.py > $O/lane_probe.log 2>&1; rc=$?; echo lane_probe=$rc; grep -v amdgpu.ids $O/lane_probe.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/md5_probe.py > $O/md5_probe.log 2>&1; rc=$?; echo md5_probe=$rc; grep -v amdgpu.ids $O/md5_probe.log | tail -6; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/md5_tlb_probe.py > $O/md5_tlb.log 2>&1; rc=$?; echo md5_tlb=$rc; grep -v amdgpu.ids $O/md5_tlb.log | tail -6
exit $rc
