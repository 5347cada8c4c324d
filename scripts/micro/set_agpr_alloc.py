#!/usr/bin/env python3
"""Set LLVM's "amdgpu-agpr-alloc" attribute on selected kernels of a device .ll file.

With AGPR-resident LU factors, LLVM by default splits a wave's unified register budget evenly
between VGPRs and AGPRs (128/128 at 2 waves/SIMD) and spills VGPRs; the attribute (no source-level
spelling in clang) reserves exactly the AGPRs the factors need and leaves the rest to VGPRs.
Usage: set_agpr_alloc.py in.ll out.ll SYMBOL_SUBSTRING=NUM_AGPRS ...
"""
import re
import sys


def main():
    src, dst, specs = sys.argv[1], sys.argv[2], [a.split("=") for a in sys.argv[3:]]
    text = open(src).read()
    lines = text.split("\n")
    groups = {m.group(1): m.group(2) for m in re.finditer(r"^attributes #(\d+) = \{(.*)\}$", text, re.M)}
    nxt = max(int(g) for g in groups) + 1
    new_groups = []
    done = []
    for i, ln in enumerate(lines):
        if not ln.startswith("define ") or "amdgpu_kernel" not in ln:
            continue
        for sub, num in specs:
            if sub not in ln.split("(")[0]:
                continue
            m = re.search(r"\) (?:[a-z_ ]*)?#(\d+)(?: [^#]*)?\{$", ln)
            if not m:
                raise SystemExit(f"no attribute group on: {ln[:160]}")
            body = re.sub(r' "amdgpu-agpr-alloc"="[^"]*"', "", groups[m.group(1)])
            body = body.replace(" nounwind ", f' nounwind "amdgpu-agpr-alloc"="{num}" ', 1)
            lines[i] = ln[:m.start(1)] + str(nxt) + ln[m.end(1):]
            new_groups.append(f"attributes #{nxt} = {{{body}}}")
            done.append((sub, num, nxt))
            nxt += 1
    if len(done) != len(specs):
        raise SystemExit(f"kernels not found: {specs} -> {done}")
    open(dst, "w").write("\n".join(lines + new_groups) + "\n")


if __name__ == "__main__":
    main()
