#!/bin/bash
# register / spill summary of the step kernels of the current sources (host tool, no GPU)
#   bash tools/isa_regs.sh [extra hipcc flags...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp /tmp/isa_XXXX.s)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-fast-math -fno-slp-vectorize --cuda-device-only -S "$@" \
  "$ROOT/mujoco_playground_amd/csrc/ackphys_step.hip" -o "$T" 2>/dev/null
python3 - "$T" <<'PY'
import collections, re, sys
s = open(sys.argv[1]).read()
for k in ("ackphys_step_nc_kernel", "ackphys_step_quad_kernel", "ackphys_step_obst_kernel",
          "ackphys_rollout_nc_kernel", "ackphys_rollout_quad_kernel", "ackphys_rollout_obst8_kernel",
          "ackphys_ppo_rollout_quad_kernel", "ackphys_ppo_rollout_obst8_kernel"):
    i = s.find("\n" + k + ":"); j = s.index(".Lfunc_end", i)
    ops = [l.split()[0] for l in s[i:j].split("\n") if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = collections.Counter(ops)
    def g(f):  # kernels that call functions report max(own, callee's)
        v = re.search(r"\.set " + k + r"\." + f + r", (.+)", s).group(1).strip()
        if v.isdigit():
            return v
        nums = [int(x) for x in re.findall(r"\b(\d+)\b", v)]
        callees = re.findall(r"(\.L\w+)\." + f, v)
        nums += [int(re.search(re.escape(c) + r"\." + f + r", (\d+)", s).group(1)) for c in callees]
        return str(max(nums)) if nums else v
    print(f"{k}: {len(ops)} instr, vgpr {g('num_vgpr')} agpr {g('num_agpr')} sgpr {g('numbered_sgpr')}, "
          f"v_mov {c['v_mov_b32_e32']}, agpr moves {c['v_accvgpr_write_b32'] + c['v_accvgpr_read_b32']}, "
          f"sgpr lane spills {c['v_readlane_b32'] + c['v_writelane_b32']}, scratch {sum(v for o, v in c.items() if o.startswith('scratch'))}, "
          f"s_nop {c['s_nop']}, lds {sum(v for o, v in c.items() if o.startswith('ds_'))}")
PY
rm -f "$T"
