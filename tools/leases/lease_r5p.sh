# round 5, lease p: pageable host path with the copy pool bound to the GPU's NUMA node vs unbound;
# host-path GPU tests
set -o pipefail
mkdir -p gpurun_out
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('gpu pci', p.pci_domain_id, p.pci_bus_id, p.pci_device_id)" 2>&1 | tail -1
for f in /sys/bus/pci/devices/*; do v=$(cat $f/vendor 2>/dev/null); c=$(cat $f/class 2>/dev/null); case "$c" in 0x0380*|0x1200*) [ "$v" = 0x1002 ] && echo "$(basename $f) node $(cat $f/numa_node)";; esac; done | head -4
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "host" > gpurun_out/r5p_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r5p_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for numa in 0 1; do
    PPFS_ECC_COPY_NUMA=$numa timeout -k 10 300 python tools/probes/host_path_probe.py --modes pageable --reps 3 --from-torch > gpurun_out/r5p_tmp.jsonl 2>gpurun_out/r5p_probe.err || { tail -5 gpurun_out/r5p_probe.err; exit 1; }
    python3 -c "import json,sys; [print(json.dumps({'numa': int(sys.argv[1]), 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $numa $r gpurun_out/r5p_tmp.jsonl >> gpurun_out/r5p_numa_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/r5p_numa_ab.jsonl'):
    d=json.loads(l); print(d['numa'], d['round'], d['op'], d['GiBps'])"
