#!/bin/bash
# (since this change the production build has PG_NT_STORE=1; the old base is -DPG_NT_STORE=0)
# round 4: non-temporal epilogue stores in the global-operand epilogues
# (diagnostic build art-sbir_amd/build_var/libntst.so, hipcc -DPG_NT_STORE=1 on
# pgemm.hip / pp256.hip) against the production build: timing and read bytes by
# request size of the fused BN-backward dgrads, tools/dgrad_bench.py shapes 3, 4, 6
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/ntst
cd /tmp && export TMPDIR=/tmp
for v in base nt; do
  if [ $v = base ]; then unset ARTSBIR_LIB; else export ARTSBIR_LIB=$R/art-sbir_amd/build_var/libntst.so; fi
  d=$R/gpurun_out/ntst/$v
  rm -rf $d
  SHAPES=3,4,6 CFGS=16,18,22 timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ --output-format csv -d $d -o run -- python3 $R/tools/dgrad_bench.py > $d.log 2>&1 || { echo "FAIL $v"; tail -5 $d.log; exit 1; }
  SHAPES=3,4,6 CFGS=16,18,22 timeout -k 10 180 python3 $R/tools/dgrad_bench.py > $d.time.log 2>&1 || { echo "FAIL time $v"; exit 1; }
  echo "== $v"; grep -v amdgpu $d.time.log
  python3 - $d $R <<'PY'
import sys, glob
sys.path.insert(0, sys.argv[2] + "/profiles")
import summarize_pmc as sp
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
for k, (n, b, nreq, rd) in sp.load_req(f).items():
    if "bnb" in k:
        print(f"  {k:45s} {n:3d} launches  read {b / n / 1e9:7.3f} GB/launch (all shapes pooled)")
PY
done
