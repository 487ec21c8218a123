set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ANISO_HM_VAR=68 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "harmonic or config3" --timeout 300 --timeout-method thread > gpurun_out/cl_tests.log 2>&1 || { tail -60 gpurun_out/cl_tests.log; exit 1; }
tail -1 gpurun_out/cl_tests.log
bash tools/ab_env.sh "ANISO_HM_VAR=4" "ANISO_HM_VAR=68" "ANISO_HM_VAR=4 ANISO_OVERLAP=0" "ANISO_HM_VAR=68 ANISO_OVERLAP=0"
ANISO_HM_VAR=68 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/xcd_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/xcd_fetch.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob,collections
a=collections.defaultdict(list)
for f in glob.glob('gpurun_out/xcd_fetch/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_m2l_hc' in r['Kernel_Name'] or 'k_near_hm' in r['Kernel_Name']: a[r['Kernel_Name'][:30]].append(float(r['Counter_Value']))
for k,v in a.items(): print(k, 'fetch GB (x2 corrected)', 2*sum(v)/len(v)*1024/1e9)
PY
