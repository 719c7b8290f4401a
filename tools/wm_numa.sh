# tools/wide_modes.py with the caller on each NUMA node of the box's allowed CPUs
set -u
cd "$GRAFT_REPO_ROOT"
lscpu | grep -i "numa node" > gpurun_out/wm_numa.txt
python3 -c "import os; print(sorted(os.sched_getaffinity(0)))" >> gpurun_out/wm_numa.txt
for node in 0 1; do
  cpus=$(python3 -c "
import os, glob
node = $node
mine = set(int(c) for c in open(glob.glob(f'/sys/devices/system/node/node{node}/cpulist')[0]).read().strip().replace('-', ' ').split() if False) if False else None
allowed = sorted(os.sched_getaffinity(0))
def nodes_of(cpu):
    return [int(p.split('node')[-1]) for p in glob.glob(f'/sys/devices/system/cpu/cpu{cpu}/node*')]
pick = [c for c in allowed if node in nodes_of(c)][:8]
print(','.join(map(str, pick)))")
  echo "node $node cpus $cpus" >> gpurun_out/wm_numa.txt
  [ -n "$cpus" ] || continue
  for ev in ${WM_ENV:-PBFTV_QC_NT=1}; do
    env "$ev" timeout -k 10 400 taskset -c "$cpus" python -u tools/${WM_TOOL:-wide_modes.py} ${WM_ARGS:-3} > "gpurun_out/wm_node${node}_$ev.jsonl" 2>&1 || exit $?
  done
done
