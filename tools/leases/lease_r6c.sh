# round 6, lease c: LDS-DMA layout probe (contiguous vs piece-major wave tiles, cfg5 decode input)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probes/dma_layout_probe.bin > gpurun_out/r6c_dma_layout.jsonl 2>&1; rc=$?
cat gpurun_out/r6c_dma_layout.jsonl; exit $rc
