#!/bin/bash
# One parameterised GPU-box script (round 4; replaces the one-off tools/gpu_*.sh lease scripts).
# Kernel-time A/Bs of one codec: tools/ab_codec.sh (tools/time_codec.py); profiles:
# tools/profile_box.sh (RS bench), tools/prof_cfg4.sh (cfg4), tools/prof_r4.sh (all three).
#   bash tools/gpu.sh TAG STEP [STEP ...]
# Steps run in order, each under its own time limit; the script stops at the first failure (a GPU
# fault, abort or time limit ends the call -- nothing is retried).  Outputs: gpurun_out/TAG_*.
#   tests[=K]    pytest -m gpu over tests/ (K: a -k expression; '+' stands for a space)
#   lifecycle    pytest -m gpu over tests/test_gpu_lifecycle.py
#   rs           the RS parity tests (tests/test_gpu_parity.py -k rs)
#   parity       every test of tests/test_gpu_parity.py (RS, CRC, Hamming, parity vs the oracle)
#   smoke        __graft_entry__.smoke()
#   bench        the default bench line (no CPU column, no host-inclusive leg)
#   benchfull    the default bench line with every leg (what the driver runs)
#   cfg5         the cfg5 (RS t = 16, 4 KiB) bench line
#   configs      tools/bench_configs.py (every BASELINE config, kernel-only)
#   prof         tools/profile_box.sh TAG (rocprofv3 kernel trace + PMC passes)
#   ab=A,B[,N]   interleaved bench A/B of two library builds (paths), N rounds (default 3)
#   tktrace      phase traces of the t <= 4 kernels (the trace build, tools/build_alt.sh)
#   lds[=ARGS]   one rocprofv3 PMC pass (SQ_LDS_IDX_ACTIVE, SQ_LDS_BANK_CONFLICT) over a short bench
#                run (ARGS: extra bench flags, '+' for a space): conflict cycles / LDS cycles per kernel
set -o pipefail
TAG=${1:?tag}
shift
mkdir -p gpurun_out
O=gpurun_out/${TAG}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('kernels_ms'), d.get('in_step_frac'))" "$1" "$2"; }
for step in "$@"; do
    case "$step" in
    tests | tests=*)
        K=${step#tests}; K=${K#=}; K=${K//+/ }
        timeout -k 10 900 $PYT tests ${K:+-k "$K"} > ${O}_pytest.log 2>&1
        rc=$?; tail -3 ${O}_pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    lifecycle)
        timeout -k 10 300 $PYT tests/test_gpu_lifecycle.py > ${O}_lifecycle.log 2>&1
        rc=$?; tail -3 ${O}_lifecycle.log; [ $rc -eq 0 ] || exit $rc ;;
    rs)
        timeout -k 10 600 $PYT tests/test_gpu_parity.py -k rs > ${O}_rs.log 2>&1
        rc=$?; tail -3 ${O}_rs.log; [ $rc -eq 0 ] || exit $rc ;;
    parity)
        timeout -k 10 900 $PYT tests/test_gpu_parity.py > ${O}_parity.log 2>&1
        rc=$?; tail -3 ${O}_parity.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
        timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1
        rc=$?; tail -2 ${O}_smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
        timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-configs > ${O}_bench.json 2> ${O}_bench.err \
            || { tail -5 ${O}_bench.err; exit 1; }
        line ${O}_bench.json bench ;;
    benchfull)
        timeout -k 10 600 python bench.py > ${O}_benchfull.json 2> ${O}_benchfull.err || { tail -5 ${O}_benchfull.err; exit 1; }
        line ${O}_benchfull.json benchfull ;;
    cfg5)
        timeout -k 10 300 python bench.py --block-size 4096 --t 16 --no-cpu-baseline --no-host-inclusive --no-configs \
            > ${O}_bench_cfg5.json 2> ${O}_bench_cfg5.err || { tail -5 ${O}_bench_cfg5.err; exit 1; }
        line ${O}_bench_cfg5.json cfg5 ;;
    configs)
        timeout -k 10 600 python tools/bench_configs.py > ${O}_configs.jsonl 2> ${O}_configs.err || { tail -5 ${O}_configs.err; exit 1; }
        cat ${O}_configs.jsonl ;;
    prof)
        timeout -k 10 900 bash tools/profile_box.sh ${TAG} --no-configs > ${O}_prof.log 2>&1 || { echo "profile failed"; tail ${O}_prof.log; exit 1; }
        tail -20 ${O}_prof.log ;;
    ab=*)
        IFS=, read -r A B N <<< "${step#ab=}"
        for r in $(seq 1 ${N:-3}); do
            for L in "$A" "$B"; do
                PPFS_ECC_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-configs \
                    > ${O}_ab.tmp 2> ${O}_ab.err || { tail -5 ${O}_ab.err; exit 1; }
                echo "{\"lib\": \"$L\", \"round\": $r, \"line\": $(tail -1 ${O}_ab.tmp)}" >> ${O}_ab.jsonl
                line ${O}_ab.tmp "$(basename $L) r$r"
            done
        done ;;
    tktrace)
        T=$PWD/paritypartyfs_amd/_lib/lease/libppfs_ecc_trace.so
        PPFS_ECC_LIB=$T timeout -k 10 120 python tools/tk_trace.py 2> /dev/null > ${O}_tktrace.jsonl || { tail ${O}_tktrace.jsonl; exit 1; }
        cat ${O}_tktrace.jsonl ;;
    lds | lds=*)
        A=${step#lds}; A=${A#=}; A=${A//+/ }
        R=/tmp/lds_${TAG}_$$; mkdir -p $R/lds
        ( cd /tmp && TMPDIR=/tmp timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT -d $R/lds -o lds \
            --output-format csv -- python3 $OLDPWD/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
            --no-configs $A ) > ${O}_lds.log 2>&1 || { tail -5 ${O}_lds.log; exit 1; }
        python3 tools/pmc_reduce.py $R ${O}_lds.json && rm -rf $R
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k, 'conflict/active %.4f' % (v['SQ_LDS_BANK_CONFLICT'] / max(v['SQ_LDS_IDX_ACTIVE'], 1)), v) for k, v in d.items() if v.get('SQ_LDS_IDX_ACTIVE')]" ${O}_lds.json ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
