#!/bin/bash
# (since this change the production build has PG_NT_STORE=1; the old base is -DPG_NT_STORE=0)
# round 4: C2 step with non-temporal global-operand epilogue stores (nt; nt2 adds the
# elementwise passes' stores, -DARTSBIR_NT_STORES=1 on elementwise.hip) (diagnostic
# build art-sbir_amd/build_var/libntst.so) against the production build,
# alternated twice on one box (C2 leg only, 10 timed steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
run() {
  case $1 in base) unset ARTSBIR_LIB ;; nt) export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libntst.so ;; nt2) export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libntst2.so ;; esac
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --no-loss-check --no-profile --steps 10 --warmup 3 > gpurun_out/ntstep.json 2> gpurun_out/ntstep.err || { echo "FAIL $1"; tail -5 gpurun_out/ntstep.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ntstep.json').read().strip().splitlines()[-1]);print('$1', d['ms_per_step'], d['value'])"
}
run base && run nt && run nt2 && run base && run nt && run nt2
