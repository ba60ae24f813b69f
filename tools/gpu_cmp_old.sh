cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/cmp
R=$PWD
(cd ab/wt && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/cmp/old -o old -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host > $R/gpurun_out/cmp/old.log 2>&1) || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cmp/new -o new -- python bench.py --steps 3 --warmup 1 --no-cpu --no-host > gpurun_out/cmp/new.log 2>&1 || exit 1
python - <<'PY'
import csv, glob
for tag in ("old", "new"):
    f = glob.glob(f"gpurun_out/cmp/{tag}/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for name in ("owner_kernel", "roots_kernel", "border4_kernel", "gather_kernel", "count4_kernel<float, 3, 0, false"):
        d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"])
        print(tag, name, [round(x) for x in d])
PY
