"""ISA gate for librafthip's hot kernels (gfx950).

Compiles the translation units of librafthip (raft-teststuff_amd/csrc/rh_abi.hip and
rh_solve_fast.hip, each with its own flags from __graft_entry__.UNITS) to device assembly and
checks every kernel:
  * no dynamic register indexing: `s_set_gpr_idx_*` or `v_movrel*` (a lane-dependent index into
    a register array, lowered with a scalar index, faulted k_qtf_hankel on the box in round 2;
    DESIGN.md §4) -> FAIL in any kernel;
  * no scratch traffic inside a streaming loop of any shipped kernel -- an innermost loop that issues
    buffer/global loads (the node loops of the solve kernels, the pair-tile loops of the QTF) --
    while one of its loads is outstanding (in_flight_scratch): a spill reload there shares
    `vmcnt` with the wave-table prefetch ring and drains it every node (k_solve_pair's first
    build lost 4x in phase A to exactly this) -> FAIL;
  * scratch instructions elsewhere (prologue, solve, member boundaries) are counted and reported.
Loops are found from the branch structure: a branch to a label that precedes it closes a loop
[label, branch]; a loop that contains no other loop is innermost; it streams if it holds a
buffer_load / global_load.

Usage: python tools/isa_check.py [--asm file.s] [--out report.txt]   (exit status 1 on FAIL)
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402  (the build's translation units and their flags)
# Every kernel of the shipped library is on some default dispatch path of rh_abi.hip (the opt-in
# kernels measured slower were moved out into tools/ubench/variants_src, built only with
# -DRH_VARIANTS), so every kernel is held to the streaming-loop rule.  The one exception is the
# general case solve k_solve_cases<NB>, the default for nw > 1024 or node tables beyond the LDS:
# a measured path whose current counts are a ratchet, so a change can only lower
# them.  No other kernel can get a ratchet: an entry here must name a k_solve_cases instantiation.
# (round 5: counted only while a load of the loop is in flight, in_flight_scratch; the ratchets
# fell from 6 / 14 / 14 / 21 to the counts below)
# Ratchets (measured counts; a kernel may only go down).  Round 6 re-measured them with the
# vector-memory counter modelled (vmcnt(N) waits, scratch reloads counted as loads):
# the general k_solve_cases<2> / <4> / <8> show 5 / 5 / 13 scratch accesses with loads in flight
# where the round-5 walk (reset only at vmcnt(0)) saw 0 / 0 / 8 -- the kernels did not change.
ALLOW = {"k_solve_cases<1>": 6, "k_solve_cases<2>": 5, "k_solve_cases<4>": 5, "k_solve_cases<8>": 13}
# the older measure beside it: scratch instructions anywhere inside a streaming loop,
# outstanding loads or not (a reload after a full drain still costs an L2 round trip).  The
# single-bin fast kernels (grids of <= 512 bins; C1-size designs, not the benched C2 / C4
# kernels, which have none) reload 14-20 values in their node loops, never with a load in flight.
ALLOW_LOOP = {"k_solve_cases<1>": 12, "k_solve_cases<2>": 14, "k_solve_cases<4>": 14, "k_solve_cases<8>": 22,
              "k_solve_lds<1, 128, true, 1>": 20, "k_solve_lds<1, 256, false, 1>": 14,
              "k_solve_lds<1, 512, false, 1>": 14}
assert all(k.startswith("k_solve_cases<") for k in ALLOW)
assert all(k.startswith(("k_solve_cases<", "k_solve_lds<1,")) for k in ALLOW_LOOP)
DYN_INDEX = re.compile(r"^\s*(s_set_gpr_idx\w*|v_movrel\w*)")
SCRATCH = re.compile(r"^\s*(scratch_|buffer_\w+.*\boff(en)?\b.*s\[0:3\])")
LABEL = re.compile(r"^(\.LBB\w+|\w+):")
BRANCH = re.compile(r"^\s*s_(cbranch_\w+|branch)\s+(\.LBB\w+)")
STREAM = re.compile(r"^\s*(buffer_load|global_load)")


def compile_asm(defines=()):
    """Device assembly of every translation unit (compiled in parallel), concatenated."""
    fd, path = tempfile.mkstemp(suffix=".s")
    os.close(fd)
    procs, parts = [], []
    for unit, flags in G.UNITS:
        part = path + "." + unit + ".s"
        parts.append(part)
        procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", *flags,
                                       *defines, "--offload-device-only", "-S", "-o", part, os.path.join(G.CSRC, unit)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    for p in procs:
        _, err = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(err.decode()[-3000:])
    with open(path, "w") as out:
        for part in parts:
            with open(part) as fh:
                out.write(fh.read())
            os.unlink(part)
    return path


def kernels(lines):
    """{mangled name: [instruction lines]} for every kernel body (up to its .Lfunc_end label)."""
    out, name, body = {}, None, []
    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m and name is None:
            name, body = m.group(1), []
            continue
        if name is not None:
            if re.match(r"^\.Lfunc_end\d+:", ln):   # the whole body: a kernel may end early in several places
                out[name] = body
                name = None
                continue
            body.append(ln)
    return out


VMCNT = re.compile(r"^\s*s_waitcnt\s+(?:.*\s)?vmcnt\((\d+)\)")
SCRATCH_LOAD = re.compile(r"^\s*(scratch_load|buffer_load\w*.*\boff(en)?\b.*s\[0:3\])")


def in_flight_scratch(body, a, b):
    """Scratch instructions of the loop [a, b] issued while one of its vector-memory loads is
    still outstanding: the hazard (a reload waits behind the ring's loads, since they share
    vmcnt, and drains it).  Walked in program order from the loop head with the vector-memory
    counter modelled: every load (wave-table stream and scratch reload alike) adds one, and
    `s_waitcnt vmcnt(N)` leaves at most N outstanding.  The loads still outstanding at the back
    edge (a prefetch ring carried into the next iteration) count as outstanding at the head.
    A scratch access once the counter is 0 -- e.g. around the LU of a bin, after its loads are
    consumed -- drains nothing.  (Straight-line walk: a branch inside the loop is followed as if
    both sides ran in order, which can only over-count.)"""
    def walk(carried):
        out, hits = carried, []
        for i in range(a, b + 1):
            ln = body[i]
            m = VMCNT.match(ln)
            if m:
                out = min(out, int(m.group(1)))
            elif SCRATCH.match(ln):
                if out > 0:
                    hits.append(i)
                if SCRATCH_LOAD.match(ln):
                    out += 1
            elif STREAM.match(ln):
                out += 1
        return out, hits
    carried, _ = walk(0)
    return walk(carried)[1]


def analyse(body):
    labels = {}
    for i, ln in enumerate(body):
        m = LABEL.match(ln)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, ln in enumerate(body):
        m = BRANCH.match(ln)
        if m and m.group(2) in labels and labels[m.group(2)] <= i:
            loops.append((labels[m.group(2)], i))
    inner = [l for l in loops if not any(o != l and l[0] <= o[0] and o[1] <= l[1] for o in loops)]
    inner = [(a, b) for a, b in inner if any(STREAM.match(body[i]) for i in range(a, b + 1))]
    dyn = [ln.strip() for ln in body if DYN_INDEX.match(ln)]
    scr = [i for i, ln in enumerate(body) if SCRATCH.match(ln)]
    scr_inner = [i for a, b in inner for i in in_flight_scratch(body, a, b)]
    scr_loop = [i for a, b in inner for i in range(a, b + 1) if SCRATCH.match(body[i])]
    return {"dyn": dyn, "scratch": len(scr), "scratch_inner": len(scr_inner), "scratch_loop": len(scr_loop),
            "loops": len(loops), "inner": len(inner)}


def demangle(n):
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--out")
    ap.add_argument("-D", action="append", default=[], help="extra preprocessor define (A/B variants)")
    args = ap.parse_args()
    path = args.asm or compile_asm(["-D" + d for d in args.D])
    with open(path) as fh:
        ks = kernels(fh.read().split("\n"))
    rows, fails = [], []
    for name, body in sorted(ks.items()):
        r = analyse(body)
        dn = demangle(name)
        hot = True
        verdict = "ok"
        if r["dyn"]:
            verdict = "FAIL dynamic register indexing: " + "; ".join(sorted(set(r["dyn"])))
        elif hot and (r["scratch_inner"] or r["scratch_loop"]):
            allow = max([v for k, v in ALLOW.items() if k in dn] or [0])
            allow_loop = max([v for k, v in ALLOW_LOOP.items() if k in dn] or [0])
            if r["scratch_inner"] > allow:
                verdict = f"FAIL {r['scratch_inner']} scratch instructions inside streaming loops (allowed {allow})"
            elif r["scratch_loop"] > allow_loop:
                verdict = (f"FAIL {r['scratch_loop']} scratch instructions anywhere in streaming loops "
                           f"(allowed {allow_loop})")
            else:
                verdict = (f"ok (ratchet: {r['scratch_inner']} <= {allow} with loads in flight, {r['scratch_loop']} <= "
                           f"{allow_loop} anywhere in streaming loops, general path)")
        if verdict.startswith("FAIL"):
            fails.append(dn)
        rows.append(f"{dn:70s} hot={int(hot)} loops={r['loops']:3d} inner={r['inner']:3d} "
                    f"scratch={r['scratch']:4d} in_flight={r['scratch_inner']:3d} in_loops={r['scratch_loop']:3d}  "
                    f"{verdict}")
    text = "# tools/isa_check.py: gfx950 device assembly of " + " + ".join(u for u, _ in G.UNITS) + "\n" + "\n".join(rows) + "\n"
    text += f"# {len(ks)} kernels, {len(fails)} failing\n"
    print(text)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(text)
    if not args.asm:
        os.unlink(path)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
