"""Generates ubench3.hip: cycle cost of candidate Viterbi step bodies on gfx950.

Design under test ("v3"): one packet per 8 lanes, 8 trellis positions per lane as four
dwords of two 16-bit halves [H = 2*metric7][pad = marker bit 7 + 7 path-history bits].
Per dword and trellis column: history shift (lshr + bfi), branch metric by v_perm from a
per-step pattern word, partner metric = constant - own (v_sub), two v_pk_add_u16, one DPP
exchange on cross-lane phases, v_pk_min_u16.  Values are garbage; only issue cost matters.
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def body(ph, nd, cross_ctrl, pk_x=True, pk_y=True):
    L = []
    M = lambda d: f"v{10 + d}"
    S = lambda d: f"v{20 + d}"
    T = lambda d: f"v{30 + d}"
    BX = lambda d: f"v{40 + d}"
    BY = lambda d: f"v{50 + d}"
    X = lambda d: f"v{60 + d}"
    Y = lambda d: f"v{70 + d}"
    SEL = lambda d: f"v{80 + 8 * ph + d}"
    for d in range(nd):
        L.append(f"v_lshrrev_b32 {S(d)}, 1, {M(d)}")
    for d in range(nd):
        L.append(f"v_bfi_b32 {T(d)}, s20, {S(d)}, {M(d)}")
    for d in range(nd):
        L.append(f"v_perm_b32 {BX(d)}, v1, v2, {SEL(d)}")
    for d in range(nd):
        L.append(f"v_sub_u32 {BY(d)}, 0x1c801c80, {BX(d)}")
    for d in range(nd):
        L.append((f"v_pk_add_u16 {X(d)}, {T(d)}, {BX(d)}" if pk_x else f"v_add_u32 {X(d)}, {T(d)}, {BX(d)}"))
    for d in range(nd):
        L.append((f"v_pk_add_u16 {Y(d)}, {T(d)}, {BY(d)}" if pk_y else f"v_add_u32 {Y(d)}, {T(d)}, {BY(d)}"))
    if cross_ctrl:
        if nd < 3:
            L.append("s_nop 1")
        for d in range(nd):
            L.append(f"v_mov_b32_dpp {Y(d)}, {Y(d)} {cross_ctrl} row_mask:0xf bank_mask:0xf")
        for d in range(nd):
            L.append(f"v_pk_min_u16 {M(d)}, {X(d)}, {Y(d)}")
    elif ph == 5:
        for d in range(nd):
            L.append(f"v_pk_min_u16 {M(d)}, {X(d)}, {Y(d)} op_sel:[0,1] op_sel_hi:[1,0]")
    else:
        for d in range(nd):
            L.append(f"v_pk_min_u16 {M(d)}, {X(d)}, {Y(d ^ (1 if ph == 4 else 2) if nd > 1 else d)}")
    return L


def kernel(name, nd, ctrls, **kw):
    lines = []
    for ph in range(6):
        lines += body(ph, nd, ctrls[ph], **kw)
    asm = "\\n\\t".join(lines)
    return f"""
__global__ __launch_bounds__(256) void {name}(uint32_t* out, uint32_t s) {{
  uint32_t r = threadIdx.x;
  asm volatile(
      "s_mov_b32 s20, 0x00ff00ff\\n\\t"
      "s_mov_b32 s21, {ITERS}\\n\\t"
      "v_mov_b32 v1, %[r]\\n\\tv_mov_b32 v2, 0x80808080\\n\\t"
      "LOOP_{name}:\\n\\t"
      "{asm}\\n\\t"
      "s_sub_u32 s21, s21, 1\\n\\t"
      "s_cmp_lg_u32 s21, 0\\n\\t"
      "s_cbranch_scc1 LOOP_{name}\\n\\t"
      "v_mov_b32 %[r], v10\\n\\t"
      : [r] "+v"(r) : : "s20", "s21", "scc", "memory",
      {", ".join(f'"v{i}"' for i in range(1, 130))});
  out[blockIdx.x * 256 + threadIdx.x] = r;
}}
"""


ITERS = 2048
K8 = ["quad_perm:[1,0,3,2]", "quad_perm:[2,3,0,1]", "row_half_mirror", None, None, None]
K4 = ["row_ror:8", "row_mirror", "quad_perm:[2,3,0,1]", "quad_perm:[1,0,3,2]", None, None]
KS = [
    ("k8_pk", 4, K8, {}, 6 * 4),
    ("k8_addx", 4, K8, {"pk_x": False, "pk_y": False}, 6 * 4),
    ("k4_pk", 2, K4, {}, 6 * 2),
]

src = ["#include <hip/hip_runtime.h>", "#include <cstdio>", "#include <cstdint>"]
for name, nd, ctrls, kw, _ in KS:
    src.append(kernel(name, nd, ctrls, **kw).replace("{ITERS}", str(ITERS)))
src.append("typedef void (*KF)(uint32_t*, uint32_t);")
src.append("int main() {")
src.append("  struct { const char* n; KF f; int dw_steps; int lanes_per_pkt; } ks[] = {" +
           ", ".join(f'{{"{n}", {n}, {dws}, {64 // (2 * nd)}}}' for n, nd, _, _, dws in KS) + "};")
src.append(r"""
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  uint32_t* out; (void)hipMalloc(&out, (size_t)cus * 16 * 256 * 4);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int wps : {1, 2, 4, 8}) {
    for (auto& k : ks) {
      const int blocks = cus * wps;
      k.f<<<blocks, 256>>>(out, 7);
      (void)hipEventRecord(a);
      k.f<<<blocks, 256>>>(out, 7);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      const double cyc = ms * 1e-3 * 2.4e9;
      const double wave_steps = (double)wps * ITERS_ * 6;          // per SIMD
      const double pkt_steps = wave_steps * (64 / k.lanes_per_pkt);
      printf("wps=%d %-10s %7.3f ms  %7.2f cyc/wave-step  %6.2f cyc/packet-step (per SIMD @2.4GHz)\n",
             wps, k.n, ms, cyc / wave_steps, cyc / pkt_steps);
      fflush(stdout);
    }
  }
  return 0;
}""".replace("ITERS_", str(ITERS)))
open(os.path.join(HERE, "ubench3.hip"), "w").write("\n".join(src))
