set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in stream new stream new; do
  lib=$R/picotcp_amd/libpicocsum.so
  [ $v != new ] && lib=$R/picotcp_amd/ab/libpicocsum_$v.so
  rm -rf $O/kt_$v
  PICO_CSUM_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o run --output-format csv -- python3 $R/bench.py --config c2 --steps 50 --warmup 5 --no-cpu --no-e2e --no-verify > $O/kt_$v.log 2>&1
  python3 - <<PY
import csv,glob,statistics
f=glob.glob("$O/kt_$v/**/run_kernel_trace.csv",recursive=True)[0]
d=[int(r["End_Timestamp"])-int(r["Start_Timestamp"]) for r in csv.DictReader(open(f)) if "csum_sorted_kernel<1" in r["Kernel_Name"]]
d.sort()
print("$v", len(d), "median", d[len(d)//2]/1e3, "min", d[0]/1e3, "p90", d[int(len(d)*0.9)]/1e3)
PY
  tail -1 $O/kt_$v.log | cut -c1-200
done
