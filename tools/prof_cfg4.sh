# round 4: cfg4 kernels -- configs leg A/B against the round-3 library (same box), then PMC passes
# (VALU / LDS / waits / HBM bytes) of the Hamming and CRC kernels on the current library
set -o pipefail
TAG=${1:-r4j}
A=$PWD/paritypartyfs_amd/_lib/alt/libppfs_ecc_r3.so
for r in 1 2; do
    for L in $A $PWD/paritypartyfs_amd/_lib/libppfs_ecc.so; do
        PPFS_ECC_LIB=$L timeout -k 10 300 python tools/bench_configs.py --only cfg4 > gpurun_out/${TAG}_cfg4_tmp.jsonl 2> gpurun_out/${TAG}_cfg4.err || { tail -5 gpurun_out/${TAG}_cfg4.err; exit 1; }
        python3 -c "import json,sys; [print(sys.argv[1], sys.argv[2], json.dumps({'lib': sys.argv[1], 'round': int(sys.argv[2]), **json.loads(l)})) for l in open(sys.argv[3])]" $(basename $L) $r gpurun_out/${TAG}_cfg4_tmp.jsonl | tee -a gpurun_out/${TAG}_cfg4_ab.txt | cut -c1-400
    done
done
timeout -k 10 400 bash tools/pmc_py.sh ${TAG}_ham $PWD/tools/run_one.py hamming 4096 5 err || exit 1
timeout -k 10 400 bash tools/pmc_py.sh ${TAG}_crc $PWD/tools/run_one.py crc || exit 1
python3 tools/pmc_table.py gpurun_out/pmc_${TAG}_ham > gpurun_out/${TAG}_ham_pmc.txt && python3 tools/pmc_table.py gpurun_out/pmc_${TAG}_crc > gpurun_out/${TAG}_crc_pmc.txt
cat gpurun_out/${TAG}_ham_pmc.txt gpurun_out/${TAG}_crc_pmc.txt
