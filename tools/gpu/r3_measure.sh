#!/bin/bash
# round-3 traffic measurement: rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in
# separate runs, autotune caches loaded so no tuning trial is counted) of each
# bench leg on its own launches -> one traffic file per leg; scan statistics
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TC=$R/gpurun_out/tune_r3m.txt
cp $R/profiles/tune_r3.txt $TC
ETC=$R/gpurun_out/tune_r3_embed.txt
CTC=$R/gpurun_out/tune_r3_c5.txt
rm -f $ETC $CTC
ARTSBIR_TUNE_CACHE=$ETC timeout -k 10 240 python -u tools/embed_pass.py > gpurun_out/embed_warm.log 2>&1 || { echo EMBED_WARM_FAILED; tail -5 gpurun_out/embed_warm.log; exit 1; }
tail -1 gpurun_out/embed_warm.log
ARTSBIR_TUNE_CACHE=$CTC timeout -k 10 300 python -u tools/c5_step.py 512 fp8 > gpurun_out/c5_warm.log 2>&1 || { echo C5_WARM_FAILED; tail -5 gpurun_out/c5_warm.log; exit 1; }
tail -1 gpurun_out/c5_warm.log
cd /tmp && export TMPDIR=/tmp
for leg in train retr embed c5; do
  mkdir -p $R/gpurun_out/pmc_$leg
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/pmc_$leg/pmc_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    rm -rf $d
    case $leg in
      train) timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-preprocess --no-profile --no-loss-check --steps 2 --warmup 1 --tune-cache $TC > $d.log 2>&1 ;;
      retr) timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py --no-cpu-baseline --no-embed --no-c5 --no-preprocess --no-profile --no-loss-check --batch 8 --steps 1 --warmup 1 > $d.log 2>&1 ;;
      embed) ARTSBIR_TUNE_CACHE=$ETC timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/tools/embed_pass.py > $d.log 2>&1 ;;
      c5) ARTSBIR_TUNE_CACHE=$CTC timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/tools/c5_step.py 512 fp8 > $d.log 2>&1 ;;
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
ARTSBIR_KNN_STAT=1 timeout -k 10 300 python -u tools/retr_leg.py > gpurun_out/r3_knn_stat.log 2>&1 || { echo RETR_FAILED; tail -5 gpurun_out/r3_knn_stat.log; exit 1; }
grep noise gpurun_out/r3_knn_stat.log
