#!/bin/bash
# round-3 traffic measurement: one bench run tunes every shape of every leg and
# writes the table (the committed profiles/tune_r3.txt the bench loads by
# default); then rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate
# runs) of each leg on its own launches with that table loaded (no tuning trial
# is counted) -> one traffic file per leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TC=$R/gpurun_out/tune_r3_all.txt
rm -f $TC
timeout -k 10 600 python -u bench.py --no-cpu-baseline --tune-cache none --tune-save $TC > gpurun_out/tune_run.json 2> gpurun_out/tune_run.err || { echo TUNE_RUN_FAILED; tail -5 gpurun_out/tune_run.err; exit 1; }
echo "table: $(wc -l < $TC) entries"
cd /tmp && export TMPDIR=/tmp
for leg in train retr embed c5; do
  mkdir -p $R/gpurun_out/pmc_$leg
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/pmc_$leg/pmc_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    rm -rf $d
    case $leg in
      train) timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-preprocess --no-profile --no-loss-check --steps 2 --warmup 1 --tune-cache $TC > $d.log 2>&1 ;;
      retr) timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py --no-cpu-baseline --no-embed --no-c5 --no-preprocess --no-profile --no-loss-check --batch 8 --steps 1 --warmup 1 --tune-cache $TC > $d.log 2>&1 ;;
      embed) ARTSBIR_TUNE_CACHE=$TC timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/tools/embed_pass.py > $d.log 2>&1 ;;
      c5) ARTSBIR_TUNE_CACHE=$TC timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/tools/c5_step.py 512 fp8 > $d.log 2>&1 ;;
    esac
    rc=$?
    [ $rc = 0 ] || { echo PMC_FAILED $leg $c rc=$rc; tail -5 $d.log; exit 1; }
    echo pmc $leg $c ok
  done
done
cd $R
python3 profiles/summarize_pmc.py gpurun_out/pmc_train gpurun_out/pmc_retr gpurun_out/r3_pmc_traffic.json &&
python3 profiles/summarize_pmc.py gpurun_out/pmc_embed gpurun_out/r3_embed_pmc_traffic.json &&
python3 profiles/summarize_pmc.py gpurun_out/pmc_c5 gpurun_out/r3_c5_pmc_traffic.json || exit 1
echo summaries done
