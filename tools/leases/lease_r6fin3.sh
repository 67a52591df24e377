# round 6, third final-build lease (after the host path direct write-back): GPU suite, smoke, the driver's bench line, rocprofv3 profiles (kernel
# trace + PMC passes) of the headline and of the cfg5 step, CRC / Hamming PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6fin3_gputest.log 2>&1; rc=$?
tail -3 gpurun_out/r6fin3_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6fin3_smoke.log 2>&1 || { tail -5 gpurun_out/r6fin3_smoke.log; exit 1; }
tail -1 gpurun_out/r6fin3_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6fin3_bench.json 2> gpurun_out/r6fin3_bench.err || { tail -5 gpurun_out/r6fin3_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6fin3_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['in_step_frac'],d['roofline']['traffic']);print({k:{kk:vv for kk,vv in v.items() if 'frac' in kk} for k,v in d['configs'].items() if isinstance(v,dict)})"
timeout -k 10 700 bash tools/profile_box.sh r6fin3_cfg5 --block-size 4096 --t 16 > gpurun_out/r6fin3_prof_cfg5.log 2>&1 || { tail -5 gpurun_out/r6fin3_prof_cfg5.log; exit 1; }
timeout -k 10 700 bash tools/profile_box.sh r6fin3 > gpurun_out/r6fin3_prof.log 2>&1 || { tail -5 gpurun_out/r6fin3_prof.log; exit 1; }
echo profiles done
timeout -k 10 400 bash tools/pmc_py.sh r6fin3_crc $PWD/tools/run_one.py crc > gpurun_out/r6fin3_pmc_crc.log 2>&1 || { tail -5 gpurun_out/r6fin3_pmc_crc.log; exit 1; }
timeout -k 10 400 bash tools/pmc_py.sh r6fin3_ham $PWD/tools/run_one.py hamming 4096 5 err > gpurun_out/r6fin3_pmc_ham.log 2>&1 || { tail -5 gpurun_out/r6fin3_pmc_ham.log; exit 1; }
python3 tools/pmc_table.py gpurun_out/pmc_r6fin3_crc > gpurun_out/r6fin3_crc_pmc.txt && python3 tools/pmc_table.py gpurun_out/pmc_r6fin3_ham > gpurun_out/r6fin3_ham_pmc.txt
echo cfg4 pmc done
