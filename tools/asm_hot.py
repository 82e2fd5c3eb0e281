"""Hot-block report of one kernel in build/asm/kcdc_kernels.s (make asm): blocks with many
v_bitop3 (the hash steps), their instruction counts and SGPR-to-VGPR-lane spill traffic."""
import re
import sys

sym = sys.argv[1] if len(sys.argv) > 1 else "_ZN4kcdc3dev23split_batch_pipe_kernelILb1EEEvNS0_9BatchArgsE"
path = sys.argv[2] if len(sys.argv) > 2 else "build/asm/kcdc_kernels.s"
L = open(path).read().split("\n")
start = next(i for i, l in enumerate(L) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(L)) if L[i].startswith(".Lfunc_end") )
blocks, cur = [], ["entry", 0, 0, 0, 0]
blocks.append(cur)
for l in L[start:end]:
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        cur = [m.group(1), 0, 0, 0, 0]
        blocks.append(cur)
        continue
    s = l.strip()
    if not s or s.startswith((";", ".")):
        continue
    cur[4] += 1
    if s.startswith("v_bitop3"):
        cur[1] += 1
    if s.startswith(("v_writelane", "v_readlane")):
        cur[2] += 1
    if s.startswith("s_"):
        cur[3] += 1
tot = sum(b[4] for b in blocks)
lanes = sum(b[2] for b in blocks)
print(f"{sym}: {len(blocks)} blocks, {tot} instructions, {lanes} lane spill ops")
for b in blocks:
    if b[1] >= 32:
        print(f"  {b[0]}: bitop3 {b[1]} lane-spill {b[2]} salu {b[3]} insts {b[4]}")
