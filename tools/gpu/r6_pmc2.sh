#!/bin/bash
# round-6 closing traffic per leg (tools/gpu/r6_pmc.sh's passes, LEGS chosen per
# call): train + retr -> r6_pmc_traffic.json (the file bench.py prices the C2 and
# retrieval legs against), c5 -> r6_c5_pmc_traffic.json, embed -> r6_embed_pmc_traffic.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LEGS="${LEGS:-train retr}" bash tools/gpu/r6_pmc.sh > gpurun_out/r6_pmc2.log 2>&1; rc=$?
tail -3 gpurun_out/r6_pmc2.log; [ $rc = 0 ] || exit 1
case " ${LEGS:-train retr} " in
  *" c5 "*) python3 profiles/summarize_pmc.py gpurun_out/pmc_c5 gpurun_out/r6_c5_pmc_traffic.json || exit 1 ;;
esac
case " ${LEGS:-train retr} " in
  *" embed "*) python3 profiles/summarize_pmc.py gpurun_out/pmc_embed gpurun_out/r6_embed_pmc_traffic.json || exit 1 ;;
esac
echo done
