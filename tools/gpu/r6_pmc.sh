#!/bin/bash
# round-6 traffic measurement with the committed autotune table
# (profiles/tune_r6.txt, loaded so a kernel name stands for the same launches
# as in the bench): rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate
# runs, and a third with the read requests by size) of each leg on its own
# launches -> one traffic file per leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TC=$R/profiles/tune_r6.txt
cd /tmp && export TMPDIR=/tmp
for leg in ${LEGS:-train}; do
  mkdir -p $R/gpurun_out/pmc_$leg
  for c in FETCH_SIZE WRITE_SIZE REQ; do
    d=$R/gpurun_out/pmc_$leg/pmc_$( [ $c = FETCH_SIZE ] && echo fetch || { [ $c = WRITE_SIZE ] && echo write || echo req; } )
    [ $c = REQ ] && c="TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ"
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
case " ${LEGS:-train} " in *" retr "*) P="gpurun_out/pmc_train gpurun_out/pmc_retr" ;; *) P="gpurun_out/pmc_train" ;; esac
case " ${LEGS:-train} " in *" train "*) python3 profiles/summarize_pmc.py $P gpurun_out/r6_pmc_traffic.json ;; esac || exit 1
echo summaries done
