#!/bin/bash
# Dev: the 1e7 host-path bench with the process bound to the GPU's NUMA node, to the other node,
# and unbound (interleaved), to see how much of the host side's box-to-box spread is placement.
# Usage: TAG=r05x bash tools/exp_numa_bench.sh
O=gpurun_out/${TAG:-numa}
bus=$(python3 -c "import torch; print(torch.cuda.get_device_properties(0).pci_bus_id)" 2>/dev/null | tail -1)
node=0
for d in /sys/bus/pci/devices/*; do
  b=$(basename $d); [ $((16#$(echo $b | cut -d: -f2))) -eq "$bus" ] || continue
  [ -f $d/class ] && grep -q "0x0380\|0x0300\|0x1200" $d/class && node=$(cat $d/numa_node) && break
done
near=$(cat /sys/devices/system/node/node$node/cpulist)
far=$(cat /sys/devices/system/node/node$((1 - node))/cpulist)
echo "gpu bus $bus node $node near $near far $far" > ${O}_numa_info.txt
for r in 1 2; do
  for m in near far unbound; do
    case $m in near) pre="taskset -c $near" ;; far) pre="taskset -c $far" ;; *) pre="" ;; esac
    $pre timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-device --steps 10 --warmup 2 > ${O}_numa_${m}_r$r.json 2>> ${O}_numa.err || exit 1
  done
done
