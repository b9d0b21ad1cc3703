"""Build phase-ablated copies of librafthip.so (tools/ubench/var_<name>.so) to attribute the
case-solve time to its phases on the GPU.  The ablated libraries give wrong answers by
construction; tools/ubench/time_solve.py only times them (per executed iteration)."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "raft-teststuff_amd", "csrc")

EDITS = {
    "qNoKay": [("rh_qtf.hip", "    if (qm(q, RH_QM_KAY, m) != 0.0) {", "    if (qm(q, RH_QM_KAY, m) == 12345.0) {")],
    "qNoNodes": [("rh_qtf.hip", "    for (int n = n0; n < n1; ++n) {\n      const rh_c128* T = wk.node", "    for (int n = n0; n < n0; ++n) {\n      const rh_c128* T = wk.node")],
    # MFMA QTF path (rh_qtf_mfma.hip) ablations
    "kNoEpi": [("rh_qtf_mfma.hip", "        if (wl) {   // waterline term (:1133-1149): Re(-i kap A) = kap Im(A)\n          sre = kap * ca[r];\n        } else {",
                "        if (true) {\n          sre = kap * (ca[r] + cbk[r]);\n        } else {")],
    "kNoMfma": [("rh_qtf_mfma.hip", "          ca = mfma64(va[s], vr[s], ca);\n          cbk = mfma64(vb[s], vr[s], cbk);",
                 "          ca[0] += va[s] * vr[s];\n          cbk[0] += vb[s] * vr[s];")],
    "kNoFinal": [("rh_qtf_mfma.hip", "  if (a1 >= n2 || a2 >= n2 || a2 < a1) return;", "  if (a1 >= -1) return;")],
    "kNoRows": [("rh_qtf_mfma.hip", "    for (int ir = rlo; ir < rhi; ++ir) {", "    for (int ir = rlo; ir < rlo; ++ir) {")],
    "gNoMfmaOps": [("rh_qtf_mfma.hip", "      p1 = mfma64(a[j].r, b[j].r, p1);\n      p2 = mfma64(a[j].i, b[j].i, p2);\n      p3 = mfma64(a[j].r + a[j].i, b[j].r + b[j].i, p3);",
                    "      p1[0] += a[j].r * b[j].r;\n      p2[0] += a[j].i * b[j].i;\n      p3[0] += a[j].r * b[j].i;")],
    "gFixedLoads": [("rh_qtf_mfma.hip", "        an[j] = ld(A + (s + 4 + j) * step);\n        bn[j] = ld(B + (s + 4 + j) * step);",
                     "        an[j] = ld(A + j * step);\n        bn[j] = ld(B + j * step);")],
    "gNoEpi": [("rh_qtf_mfma.hip", "    if ((w1 != w2) && (k1 > 0) && (k2 > 0)) {   // second-order potential (raft/helpers.py:254-291)\n      const double kx = k1 * cb - k2 * cb",
                "    if (w1 < -1.0) {\n      const double kx = k1 * cb - k2 * cb")],
    "gNoPot": [("rh_qtf_mfma.hip", "  cgemm_steps(wk.Lp + ", "  if (nk < 0) cgemm_steps(wk.Lp + ")],
    "gNoMain": [("rh_qtf_mfma.hip", "  if (nk > 0)\n    cgemm_steps(", "  if (nk < 0)\n    cgemm_steps(")],
    "prof": [],          # unmodified source built with -DRH_PROF (phase cycle counters)
    # nw <= 256 (C4): 128 threads x 2 bins per lane instead of 256 x 1 (half the reductions per bin)
    "c4nb2": [("rh_abi.hip", "    const int nb = nw <= rh::kLT ? 1 : 2;\n", "    const int nb = (nw <= rh::kLT && nw > rh::kLT / 2) ? 1 : 2;\n"),
              ("rh_abi.hip", "    const int lt = nw <= rh::kLT / 2 ? rh::kLT / 2 : rh::kLT;",
               "    const int lt = nw <= rh::kLT / 2 ? rh::kLT / 4 : rh::kLT;"),
              ("rh_abi.hip", "      if (lt < rh::kLT) hipLaunchKernelGGL((rh::k_solve_lds<1, rh::kLT / 2>), grid, block, lsm, s, a);",
               "      if (lt < rh::kLT) hipLaunchKernelGGL((rh::k_solve_lds<2, rh::kLT / 4>), grid, block, lsm, s, a);")],
    # phase C: the node's drag coefficients read from LDS one node ahead (registers)
    "cPrefA": [("        int m = 0, mnext = nn > 0 ? mstart[1] : 0;\n",
                "        int m = 0, mnext = nn > 0 ? mstart[1] : 0;\n"
                "        double Ac0 = al[0], Ac1 = al[1], Ac2 = al[2], Ac3 = al[3], Ac4 = al[4];\n"),
               ("          const double* A = al + 5 * n;\n"
                "          const double A0 = A[0], A1 = A[1], A2 = A[2], A3 = A[3], A4 = A[4];\n",
                "          const double A0 = Ac0, A1 = Ac1, A2 = Ac2, A3 = Ac3, A4 = Ac4;\n"
                "          const double* An = al + 5 * (n + 1 < nn ? n + 1 : n);\n"
                "          Ac0 = An[0]; Ac1 = An[1]; Ac2 = An[2]; Ac3 = An[3]; Ac4 = An[4];\n")],
    "noLU": [("      my_sing |= !lu_solve<6>(Z, F);", "      F[0] = add(F[0], Z[0][0]);")],
    "stXo": [("        st_nt(Xo + c * nw + b, x);", "        st(Xo + c * nw + b, x);")],
    "noXo": [("        st_nt(Xo + c * nw + b, x);", "        if (x.r == 1234.5) st(Xo + c * nw + b, x);")],
    "qNoPot": [("rh_qtf.hip", "    if (pot_on && rz <= 0) {", "    if (pot_on && rz <= -1e300) {")],
    "qNoKY": [("rh_qtf.hip", "    for (int ir = NWV - 1 - wv; ir < q.nkr; ir += NWV) {", "    for (int ir = NWV - 1 - wv; ir < 0; ir += NWV) {")],
    "qNoRot": [("rh_qtf.hip", "    // (5) Rainey body-rotation terms (:1556-1575)\n    cd fr[3];\n    {", "    // (5) Rainey body-rotation terms (:1556-1575)\n    cd fr[3] = {vA[0], vA[1], vA[2]};\n    if (rz < -1e300) {")],
    "qKyUnroll": [("rh_qtf.hip", "#pragma unroll 1\n        for (int nn = 0; nn <= 10; ++nn) s = add(s, kay_omega(D1, D2, nn));",
                   "#pragma unroll\n        for (int nn = 0; nn <= 10; ++nn) s = add(s, kay_omega(D1, D2, nn));"),
                  ("rh_qtf.hip", "#pragma unroll 1\n        for (int nn = 0; nn <= 10; ++nn) s = add(s, scl(kay_omega",
                   "#pragma unroll\n        for (int nn = 0; nn <= 10; ++nn) s = add(s, scl(kay_omega")],
    "qKyUnroll4": [("rh_qtf.hip", "#pragma unroll 1\n        for (int nn = 0; nn <= 10; ++nn) s = add(s, scl(kay_omega",
                   "#pragma unroll 4\n        for (int nn = 0; nn <= 10; ++nn) s = add(s, scl(kay_omega")],
    "noA": [("      for (int n = 0; n < nn; n += 3) {\n        step(KA, n);\n        if (n + 1 < nn) step(KB, n + 1);",
             "      for (int n = 0; n < 0; n += 3) {\n        step(KA, n);\n        if (n + 1 < nn) step(KB, n + 1);")],
    "noC": [("        for (int n = 0; n < nn; n += 3) {\n          step(KA, n);",
             "        for (int n = 0; n < 0; n += 3) {\n          step(KA, n);")],
}


def build(name, edits, flags=()):
    tmp = tempfile.mkdtemp()
    dst = os.path.join(tmp, "csrc")
    shutil.copytree(CSRC, dst)
    inc = os.path.join(tmp, "..", "include")
    for e in edits:
        fname, a, b = e if len(e) == 3 else ("rh_solve.hip", e[0], e[1])
        p = os.path.join(dst, fname)
        s = open(p).read()
        assert a in s, (name, a[:60])
        s = s.replace(a, b)
        open(p, "w").write(s)
    # rh_device.h includes ../../include/rafthip.h relative to csrc
    os.makedirs(os.path.join(tmp, "x"), exist_ok=True)
    shutil.move(dst, os.path.join(tmp, "x", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    out = os.path.join(ROOT, "tools", "ubench", f"var_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                    "-Wno-unused-result", *flags, "-o", out, os.path.join(tmp, "x", "csrc", "rh_abi.hip")], check=True)
    shutil.rmtree(tmp)
    print("built", out)


if __name__ == "__main__":
    names = sys.argv[1:] or list(EDITS)
    for n in names:
        base = n[:-5] if n.endswith("+prof") else n
        build(n.replace("+", "_"), EDITS[base], ["-DRH_PROF"] if (n == "prof" or n.endswith("+prof")) else [])
