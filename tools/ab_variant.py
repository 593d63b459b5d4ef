"""Timing-only library variants, built from patched copies of csrc/ (the production sources stay
free of diagnostic switches):  python tools/ab_variant.py NAME [NAME ...]  ->  lib/libmarf_ab_NAME.so

  nodma          k_step2 without its weight-ring DMA pieces (the ring keeps whatever the slots
                 held): what the step kernel costs without streaming its weight program
  nosave         k_step2 without its saved-tensor stores (feat_l, dz_l) and their vmcnt accounting
  nodma_nosave   both
  tilenosave     the tile kernels without their saved-tile stores (C5)

  dmant / stnt / stsc1 / dmant_stnt   cache-policy bits on the weight DMA / the saved-tensor stores
                 (correct results, the same bits)

The first three compute wrong results on purpose: bench them with MARF_AB_TIMING_ONLY=1 and
MARF_LIB=<the .so> (bench.py then never reports the line as a headline)."""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd")
sys.path.insert(0, PKG)

DMA_ASM = ('asm volatile("s_mov_b32 %0, m0\\n\\ts_mov_b32 m0, %2\\n\\ts_nop 0\\n\\tglobal_load_lds_dwordx4 %1, off offset:%3\\n\\ts_mov_b32 m0, %0"\n'
           '                     : "=&s"(keep)\n'
           '                     : "v"(va), "s"(m), "n"((j & 3) * 1024)\n'
           '                     : "memory");')
SAVE = ("        s2_st16o<0>(blk, contig(f0));\n"
        "        s2_st16o<1024>(blk, contig(f1));\n"
        "        st_cur += 2;\n")

PATCHES = {
    "nodma": [("marf_step2.hip", DMA_ASM, "(void)va; (void)m; keep = 0; (void)keep;")],
    "nosave": [("marf_step2.hip", SAVE, "        (void)blk; (void)f0; (void)f1; (void)contig;\n")],
}
PATCHES["nodma_nosave"] = PATCHES["nodma"] + PATCHES["nosave"]
# the tile kernels (k_mlp_step / k_mlp_fwd / k_mlp_bwd) without their saved-tile stores: what the
# stores and the loads queued behind them (vmcnt retires in issue order) cost C5
PATCHES["tilenosave"] = [("marf_gemm.h", "    if (st.active) st.flush(act);\n}", "    (void)st;\n}")]
# cache-policy variants (correct results, same bits): the weight-ring DMA and / or the saved-tensor
# stores with the nt (streaming) or sc1 (write-through) policy bits
DMA_OP = "global_load_lds_dwordx4 %1, off offset:%3"
ST_OP = "global_store_dwordx4 %0, %1, off offset:%2"
PATCHES["dmant"] = [("marf_step2.hip", DMA_OP, DMA_OP + " nt")]
PATCHES["stnt"] = [("marf_step2.hip", ST_OP, ST_OP + " nt")]
PATCHES["stsc1"] = [("marf_step2.hip", ST_OP, ST_OP + " sc1")]
PATCHES["dmant_stnt"] = PATCHES["dmant"] + PATCHES["stnt"]


def build(name):
    import build_lib
    with tempfile.TemporaryDirectory() as td:
        pkg = os.path.join(td, "pkg")
        shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(pkg, "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(td, "include"))  # (csrc includes ../../include)
        for fn, old, new in PATCHES[name]:
            p = os.path.join(pkg, "csrc", fn)
            src = open(p).read()
            if src.count(old) != 1:
                raise SystemExit(f"{name}: patch target not found exactly once in {fn}")
            open(p, "w").write(src.replace(old, new))
        # compile the patched copy with the production flags (build_lib reads csrc/ next to HERE)
        here = build_lib.HERE
        try:
            build_lib.HERE = pkg
            build_lib._compile(os.path.join(PKG, "lib", f"libmarf_ab_{name}.so"), [], True)
        finally:
            build_lib.HERE = here


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
