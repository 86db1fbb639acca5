#!/bin/bash
# round 5: the GLB epilogue with pixel tiles outside and channel pairs inside
# (pg_epilogue_glb) against the round-4 order (PG_GLB_OLD build): parity tests of
# the fused dgrads, the C2 step with each, and the PMC read/write bytes per launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_fused_gpu.py tests/test_pgemm_gpu.py tests/test_fold_gpu.py tests/test_c2_gpu.py > gpurun_out/r5_glb_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r5_glb_tests.log; [ $rc = 0 ] || exit 1
B="python -u bench.py --no-cpu-baseline --no-c5 --no-embed --no-retrieval --no-preprocess --steps 10 --warmup 3"
OLD=$R/art-sbir_amd/build_var/libartsbir_glbold.so
timeout -k 10 400 $B > gpurun_out/r5_glb_new.json 2> gpurun_out/r5_glb_new.err || { echo BENCH_NEW_FAILED; tail -20 gpurun_out/r5_glb_new.err; exit 1; }
ARTSBIR_LIB=$OLD timeout -k 10 400 $B > gpurun_out/r5_glb_old.json 2> gpurun_out/r5_glb_old.err || { echo BENCH_OLD_FAILED; tail -20 gpurun_out/r5_glb_old.err; exit 1; }
if [ -n "$LAYOUT" ]; then
  ARTSBIR_PG_DBG=16 timeout -k 10 900 $T tests/test_fused_gpu.py tests/test_pgemm_gpu.py > gpurun_out/r5_glb_tests16.log 2>&1; rc=$?
  echo "layout tests rc=$rc"; tail -3 gpurun_out/r5_glb_tests16.log; [ $rc = 0 ] || exit 1
  ARTSBIR_PG_DBG=16 timeout -k 10 400 $B > gpurun_out/r5_glb_lay.json 2> gpurun_out/r5_glb_lay.err || { echo BENCH_LAY_FAILED; tail -20 gpurun_out/r5_glb_lay.err; exit 1; }
  python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r5_glb_lay.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("lay", d["value"], d["ms_per_step"], r.get("streams_kernel_ms"))
for k, v in r["per_kernel"].items():
    if "glb" in k:
        print(f"   {k:42s} {v['launches']/d['steps']:5.1f}/step {v['avg_us']:8.1f}us {v['share_s']*1e3/d['steps']:7.2f}ms/step")
PY
  [ -n "$NOPMC" ] && exit 0
fi
TC=$R/profiles/tune_r5.txt
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$R/gpurun_out/pmc_glb_$v/pmc_$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    rm -rf $d; mkdir -p $(dirname $d)
    if [ $v = old ]; then export ARTSBIR_LIB=$OLD; else unset ARTSBIR_LIB; fi
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d -o run -- python3 $R/bench.py --no-cpu-baseline --no-retrieval --no-embed --no-c5 --no-preprocess --no-profile --no-loss-check --steps 2 --warmup 1 --tune-cache $TC > $d.log 2>&1
    rc=$?
    [ $rc = 0 ] || { echo PMC_FAILED $v $c rc=$rc; tail -5 $d.log; exit 1; }
    echo pmc $v $c ok
  done
done
unset ARTSBIR_LIB
cd $R
python3 - <<'PY'
import json
for n in ("new", "old"):
    d = json.loads(open(f"gpurun_out/r5_glb_{n}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(n, d["value"], d["ms_per_step"], r.get("streams_kernel_ms"))
    for k, v in r["per_kernel"].items():
        if "glb" in k or "bnb" in k:
            print(f"   {k:42s} {v['launches']/d['steps']:5.1f}/step {v['avg_us']:8.1f}us {v['share_s']*1e3/d['steps']:7.2f}ms/step")
PY
for v in new old; do python3 profiles/summarize_pmc.py gpurun_out/pmc_glb_$v gpurun_out/r5_glb_pmc_$v.json > /dev/null 2>&1 || echo "summarize $v failed"; done
python3 - <<'PY'
import json
for n in ("new", "old"):
    try:
        d = json.load(open(f"gpurun_out/r5_glb_pmc_{n}.json"))
    except Exception as e:
        print(n, "no summary", e); continue
    tot = 0
    for k, v in d["kernels"].items():
        tot += v["hbm_bytes_per_launch"] * v["launches"]
    print(n, "total GB per step", round(tot / 3 / 1e9, 1))
    for k, v in d["kernels"].items():
        if "glb" in k or "bnb" in k:
            print(f"   {k:42s} {v['launches']:4d} {v['fetch_bytes_per_launch']/1e9:7.3f} GB read {v['write_bytes_per_launch']/1e9:7.3f} GB write")
PY
