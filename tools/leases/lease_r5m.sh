# round 5, lease m: what the 1-error decodes' extra time is (tools/probes/wb_probe.py), on the shipped build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/probes/wb_probe.py > gpurun_out/r5m_wb_probe.jsonl 2> gpurun_out/r5m_wb_probe.err || { tail -5 gpurun_out/r5m_wb_probe.err; exit 1; }
cat gpurun_out/r5m_wb_probe.jsonl
