# one-off diagnostic (round 4): which change made the t <= 4 kernels slower
set -o pipefail
mkdir -p gpurun_out
A=$PWD/paritypartyfs_amd/_lib/alt
NEW=$PWD/paritypartyfs_amd/_lib/libppfs_ecc.so
run() { # tag lib [env]
    env $3 PPFS_ECC_LIB=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-configs \
        > gpurun_out/r4e_$1.json 2> gpurun_out/r4e_$1.err || { tail -5 gpurun_out/r4e_$1.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['kernels_ms'], d['standalone']['encode_ms_median'], d['standalone']['clean_decode_ms_median'])" gpurun_out/r4e_$1.json $1
}
run r3 $A/libppfs_ecc_r3.so
run new $NEW
run noorder $NEW PPFS_ECC_NO_ORDER=1
run sched0 $A/libppfs_ecc_sched0.so
PPFS_ECC_LIB=$A/libppfs_ecc_trace.so timeout -k 10 120 python tools/tk_trace.py 2> /dev/null > gpurun_out/r4e_tktrace.jsonl || { tail gpurun_out/r4e_tktrace.jsonl; exit 1; }
cat gpurun_out/r4e_tktrace.jsonl
