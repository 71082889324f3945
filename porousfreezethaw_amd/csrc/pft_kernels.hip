// pft_kernels.hip -- hand-written HIP kernels for gfx950 (MI355X) + the pft_hip_* C-ABI shim.
//
// The hot path of RK_MPI_SA_solve (RK_MPI_SAsolver_hybrid2.c:351-766) with the intertrack
// right-hand side (equation.c:566-884) fused per Merson stage: each stage is ONE kernel that
// evaluates the 7-point RHS at a cell and immediately applies that stage's pointwise combine
// (hybrid2.c:378-450), the error norm (:507-524) and the candidate update (:657-668).  Every
// floating-point operation is the reference's, in the reference's order, with contraction
// disabled (-ffp-contract=off and the pragma below), so results are bit-identical to the CPU
// reference for calc_mode 0/1/10/11 (mode 2 differs only through device cosh, <= 1 ulp).
//
// Memory: per slab, a field is (n3+2) planes of n1*n2 doubles (one ghost plane each side, filled
// only at slab interfaces) between two far ghost planes (the pair kernels' two-plane halo).  Mirror / Dirichlet walls (equation.c:113-263) are folded into the
// neighbour selection: the first mirrored ghost equals the boundary cell itself.
//
// Launch geometry: a 256-thread workgroup owns 256 consecutive (i,j) columns of the flattened
// plane (fully coalesced 2 KiB loads) and marches `kz` planes in z with the z-neighbours of all
// three fields in registers (2.5-D blocking).  x/y neighbours come from the L1/L2; the linear
// workgroup id is remapped so that the 8 XCDs each take a contiguous run of tiles (their y
// neighbours then share the XCD's L2, cdna_hip_programming.md T1).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <vector>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pft_frontend.h"
#include "../../include/pft_hip.h"
#include "pft_ic_ops.h"
#include "pft_tanh.h"

#pragma clang fp contract(off)

#define PFT_BLOCK 256      // threads per workgroup of the cache kernel (merson_stage)
#define PFT_FBLOCK 256     // ... of the fused stage kernel (merson_fused).  A/B: 512 (25 x 20-pair
                           // tiles, a third fewer halo loads) measured 3-5% slower at 400^3 -- one
                           // workgroup per CU where 256 fit two to four
#define PFT_TRING 8
#define PFT_PUB_SLOTS 64

static __thread char g_err[256];

static int fail(hipError_t e, const char* what)
{
  snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
  // the failed call also left e as the thread's "last error": reset it, or the next launch's
  // hipGetLastError() check would report it again (e.g. after an allocation that found the HBM full)
  (void)hipGetLastError();
  return -(int)e - 1000;
}
#define HIPCHK(x)                                  \
  do {                                             \
    hipError_t e_ = (x);                           \
    if (e_ != hipSuccess) return fail(e_, #x);     \
  } while (0)

// ------------------------------------------------------------------------------------------
// model arithmetic (equation.c:330-421, 650-731, 835-874), operation order preserved

struct Col {           // one field at a cell: centre and its 6 face neighbours
  double c, xm, xp, ym, yp, zm, zp;
};

__device__ __forceinline__ double lam_of(const pft_consts& c, double p, double g)
{
  return g * c.lam_g + (1.0 - g) * (p * c.lam_i + (1.0 - p) * c.lam_w);
}

__device__ __forceinline__ double sshape(const pft_consts& c, double x)
{
  if (x <= c.p_eps0) return 0.0;
  if (x >= c.p_eps1) return 1.0;
  x -= c.p_eps0;
  return x * x * (c.e23 - c.e32 * x);
}

// K (du, dp) at one cell; dgl is identically 0 (equation.c:731,874)
template <int MODE>
__device__ __forceinline__ void rhs_cell(const pft_consts& c, const Col& u, const Col& p, const Col& g,
                                         double un, double& du, double& dp)
{
  // un = u + u_noise (equation.c:676,687); only the reaction terms see the noise
  const double pc = p.c, gc = g.c, uc = u.c;
  const double rho = gc * c.rho_g + (1.0 - gc) * (pc * c.rho_i + (1.0 - pc) * c.rho_w);
  const double cp = gc * c.cp_g + (1.0 - gc) * (pc * c.cp_i + (1.0 - pc) * c.cp_w);
  const double wi = fmax(0.0, 1.0 - c.zeta * gc);
  if (MODE == 10 || MODE == 11) {
    du = 0.0;
  }
  double flux = 0.0;
  if (MODE != 10 && MODE != 11) {
    const double lxm = lam_of(c, 0.5 * (p.xm + pc), 0.5 * (g.xm + gc));
    const double lxp = lam_of(c, 0.5 * (pc + p.xp), 0.5 * (gc + g.xp));
    const double lym = lam_of(c, 0.5 * (p.ym + pc), 0.5 * (g.ym + gc));
    const double lyp = lam_of(c, 0.5 * (pc + p.yp), 0.5 * (gc + g.yp));
    const double lzm = lam_of(c, 0.5 * (p.zm + pc), 0.5 * (g.zm + gc));
    const double lzp = lam_of(c, 0.5 * (pc + p.zp), 0.5 * (gc + g.zp));
    flux = c.h1_2 * (-lxm * (-u.xm + uc) + lxp * (-uc + u.xp)) +
           c.h2_2 * (-lym * (-u.ym + uc) + lyp * (-uc + u.yp)) +
           c.h3_2 * (-lzm * (-u.zm + uc) + lzp * (-uc + u.zp));
  }
  if (MODE == 2) {
    const double ch = cosh(c.gamma * (uc - c.u_star));
    const double dpdu = (c.mhg / (ch * ch)) * wi;
    const double d = flux / (rho * (cp - c.L * dpdu));
    du = d;
    dp = dpdu * d;
  } else {
    double dpdt = c.h1_2 * (-(-p.xm + pc) + (-pc + p.xp)) +
                  c.h2_2 * (-(-p.ym + pc) + (-pc + p.yp)) +
                  c.h3_2 * (-(-p.zm + pc) + (-pc + p.zp));
    if (MODE == 0 || MODE == 10) {
      const double v1 = c.h1d2 * (-p.xm + p.xp);
      const double v2 = c.h2d2 * (-p.ym + p.yp);
      const double v3 = c.h3d2 * (-p.zm + p.zp);
      const double gn = sqrt(v1 * v1 + v2 * v2 + v3 * v3) + 1E-10;
      dpdt += c.xi2a * pc * (1.0 - pc) * (pc - 0.5) - c.bam * gn * (un - c.u_star);
    } else {
      dpdt += c.xi2a * pc * (1.0 - pc) * (pc - 0.5) -
              c.sam * sshape(c, pc) * sshape(c, 1.0 - pc) * fmax(pc * (1.0 - pc), 0.0) * (un - c.u_star);
    }
    dpdt /= c.alpha;
    dpdt *= wi;
    dp = dpdt;
    if (MODE == 0 || MODE == 1) du = (flux / rho + c.L * dpdt) / cp;
  }
}

// The same arithmetic with face reuse: a face shared by two cells computed by one thread is
// evaluated once.  Across the face between cells a (minus side) and b (plus side) the reference
// computes, at a: lp * (-u_a + u_b) with lp = lambda(0.5*(p_a+p_b), 0.5*(g_a+g_b)), and at b:
// (-lm) * (-u_a + u_b) with lm = lambda(0.5*(p_a+p_b), ...) -- the same operands in the same
// order, so lm == lp and (-lm)*d == -(lp*d) exactly; likewise the Laplacian difference
// (-p_a + p_b).  FaceT carries {lp*d, -p_a + p_b} from a to b.
struct FaceT {
  double prod, dp;
};

__device__ __forceinline__ FaceT face_of(const pft_consts& c, double pa, double ga, double ua, double pb, double gb,
                                         double ub, bool need_flux)
{
  FaceT f;
  f.dp = -pa + pb;
  f.prod = need_flux ? lam_of(c, 0.5 * (pa + pb), 0.5 * (ga + gb)) * (-ua + ub) : 0.0;
  return f;
}

// rhs_cell with the x-minus and z-minus faces given (fxm, fzm: the plus faces of the neighbours),
// returning this cell's x-plus and z-plus faces
template <int MODE>
__device__ __forceinline__ void rhs_cell_f(const pft_consts& c, const Col& u, const Col& p, const Col& g, double un,
                                           const FaceT& fxm, const FaceT& fzm, FaceT& fxp, FaceT& fzp, double& du,
                                           double& dp)
{
  constexpr bool FLUX = MODE != 10 && MODE != 11;
  const double pc = p.c, gc = g.c, uc = u.c;
  const double rho = gc * c.rho_g + (1.0 - gc) * (pc * c.rho_i + (1.0 - pc) * c.rho_w);
  const double cp = gc * c.cp_g + (1.0 - gc) * (pc * c.cp_i + (1.0 - pc) * c.cp_w);
  const double wi = fmax(0.0, 1.0 - c.zeta * gc);
  fxp = face_of(c, pc, gc, uc, p.xp, g.xp, u.xp, FLUX);
  fzp = face_of(c, pc, gc, uc, p.zp, g.zp, u.zp, FLUX);
  if (MODE == 10 || MODE == 11) du = 0.0;
  double flux = 0.0;
  if (FLUX) {
    const double lym = lam_of(c, 0.5 * (p.ym + pc), 0.5 * (g.ym + gc));
    const double lyp = lam_of(c, 0.5 * (pc + p.yp), 0.5 * (gc + g.yp));
    flux = c.h1_2 * (-fxm.prod + fxp.prod) +
           c.h2_2 * (-lym * (-u.ym + uc) + lyp * (-uc + u.yp)) +
           c.h3_2 * (-fzm.prod + fzp.prod);
  }
  if (MODE == 2) {
    const double ch = cosh(c.gamma * (uc - c.u_star));
    const double dpdu = (c.mhg / (ch * ch)) * wi;
    const double d = flux / (rho * (cp - c.L * dpdu));
    du = d;
    dp = dpdu * d;
  } else {
    double dpdt = c.h1_2 * (-fxm.dp + fxp.dp) +
                  c.h2_2 * (-(-p.ym + pc) + (-pc + p.yp)) +
                  c.h3_2 * (-fzm.dp + fzp.dp);
    if (MODE == 0 || MODE == 10) {
      const double v1 = c.h1d2 * (-p.xm + p.xp);
      const double v2 = c.h2d2 * (-p.ym + p.yp);
      const double v3 = c.h3d2 * (-p.zm + p.zp);
      const double gn = sqrt(v1 * v1 + v2 * v2 + v3 * v3) + 1E-10;
      dpdt += c.xi2a * pc * (1.0 - pc) * (pc - 0.5) - c.bam * gn * (un - c.u_star);
    } else {
      dpdt += c.xi2a * pc * (1.0 - pc) * (pc - 0.5) -
              c.sam * sshape(c, pc) * sshape(c, 1.0 - pc) * fmax(pc * (1.0 - pc), 0.0) * (un - c.u_star);
    }
    dpdt /= c.alpha;
    dpdt *= wi;
    dp = dpdt;
    if (MODE == 0 || MODE == 1) du = (flux / rho + c.L * dpdt) / cp;
  }
}

// ------------------------------------------------------------------------------------------
// the fused stage kernel

struct StageArgs {
  const double* in;    // stage input state (u, p, gl)
  const double* x;     // solution x
  const double* k1;
  const double* k3;
  const double* k4;
  double* kout;        // K of this stage (stages 0, 1, 3, 4)
  double* out;         // next stage input (1..4) or candidate x(t+h) (5)
  unsigned long long* eps_bits;
  unsigned int* nonfinite;
  const double* noise; // u_noise [k][j][i] or null (u_noise_amp == 0)
  long fs;             // field stride (doubles)
  int n1, n2, n3, plane;
  int has_below, has_above;
  int k_begin, k_end, kz, ntile, nchunk;
  int kspan;           // planes a chunk processes from its start (kz, or 1 for the boundary planes)
  // inline boundary (merson_fused; as PairArgs): the first nbw workgroups produce the planes the
  // exchange sends and count themselves in *bdone; bends 1: the first and last chunk of every tile
  // column, 0: two-plane chunks at each end; the other nint workgroups run chunks c0 ..
  int nbw, bends, c0, nint;
  unsigned long long* bdone;
  double T_top;        // Dirichlet value T_top(t_stage), equation.c:110
  double coef, h;
  double em0, em1, em2;
  // recompute path (merson_fused): the stage input is rebuilt from x and the K's
  const double* k2;    // K2 (stored only on this path; the reference aliases it with K3)
  double cin;          // coefficient of the stage-input combine: h3, h6, h8, h for stages 2..5
  int gwx, gty;        // merson_fused tile: gwx cell pairs x gty rows (fused_geometry)
  int gl_keep;         // stage 5: x(t+h) of gl is not stored, XN already holds it (pft_slab_set_gl_keep)
  // stage 5 (merson_fused): the last workgroup to finish publishes the error norm straight to
  // pinned host memory (pub[0] eps bits, pub[1] non-finite flag, both pre-set to a sentinel by
  // the host) and resets the accumulator; pub_count counts the finished workgroups
  unsigned long long* pub;
  unsigned int* pub_count;
  struct EpsShard* shards;   // stage 5: the error norm's per-shard accumulators (eps_arrive)
  // deferred publication (eps_reduce_publish): stage 5 stores its workgroups' partials to part;
  // stage 1 with npart > 0 reduces npart partials in its last workgroup and publishes them to pub
  unsigned long long* part;
  int npart;
  // Gated step (f4, small slabs, pft_slab_gate_*): this launch was enqueued before the step it
  // belongs to was decided.  gate -> 3 device words the previous speculative stage 1 wrote with
  // its decision (gate_decide): [0] a sequence number (the launch runs iff == gseq; the skip bit
  // never equals it), [1] t, [2] h of the step (bit patterns): the launch derives its scalars
  // from them with the solver's own expressions (gate_scalars).
  const unsigned long long* gate;
  unsigned long long gseq;
  // ... and the decision: the speculative stage 1's extra workgroup, once it has the error norm,
  // decides the step as hybrid2.c:578-611 does and writes it to gdev (for the launches gated on
  // it) and to pinned gpin (for the host, which takes its own decision and compares bit for bit).
  // gdec_seq: its sequence number; dt, dh: t and h of the step being decided (a gated launch
  // takes them from its gate); the solve's constants: final time, delta, h_min, delta_mode ==
  // DELTA_LOCAL, handle_nan.
  unsigned long long* gdev;
  unsigned long long* gpin;
  unsigned long long gdec_seq;
  double dt, dh, d_final, d_delta, d_hmin;
  int d_local, d_nan;
  int d_flip;          // test hook (env PFT_GATE_FLIP = N): every N-th accepted decision leaves the
                       // device with the last bit of its h flipped, so the host's check must discard
                       // and relaunch that step (tests/test_gate_gpu.py)
};

#define PFT_GATE_SKIP (1ULL << 63)
#define PFT_GATE_SLOTS 64

// the scalars of a gated launch from the decided (t, h), exactly as rk_solver.c's run_fused and
// run_stage form them (hybrid2.c:355: h/2.0, h/3.0, h/6.0, h/8.0; the stage times t + h3, t + h2,
// t + h; equation.c:110 T_top; the stage-input coefficients h/3.0, h/6.0, h/8.0, h).  IEEE
// division and addition are correctly rounded on both sides (-ffp-contract=off): the same bits.
template <int STAGE>
__device__ __forceinline__ void gate_scalars(StageArgs& a, const pft_consts& c, double t, double h)
{
  const double h2 = h / 2.0, h3 = h / 3.0, h6 = h / 6.0, h8 = h / 8.0;
  double ts = t + h;
  if (STAGE == 1) {                      // the speculative stage 1 of the next step (coef 0, h 0)
    a.coef = 0.0;
    a.h = h;
    a.cin = h;
  } else {
    ts = STAGE <= 3 ? t + h3 : (STAGE == 4 ? t + h2 : t + h);
    a.coef = STAGE == 2 ? h6 : (STAGE == 3 ? h8 : (STAGE == 4 ? h : h3));
    a.h = h;
    a.cin = STAGE == 2 ? h / 3.0 : (STAGE == 3 ? h / 6.0 : (STAGE == 4 ? h / 8.0 : h));
  }
  a.T_top = ts < c.phase_switch_time ? c.top_temp1 : c.top_temp2;
  if (STAGE == 5) a.gl_keep = a.gl_keep && isfinite(a.coef);
}

// x^0.2 rounded to nearest, for the step-size control.  glibc's pow (the host's) rounds correctly
// but for rare hard cases; ocml's is within ~1 ulp (10% of the decisions differed in the last
// bit).  So the candidate c = pow(x, 0.2) is checked against the midpoints to its neighbours in
// double-double arithmetic: v = x^0.2 > m  <=>  x > m^(1/0.2), and 1/0.2 = 5 / (1 + 5 e) with
// 0.2 = 1/5 + e, e = 2^-54 / 5, so m^(1/0.2) = m^5 (1 - 25 e ln m) to far below the ~2^-53 the
// comparison needs.  Outside a safe range the candidate stays (the host's check catches it).
struct pft_dd {
  double hi, lo;
};
__host__ __device__ __forceinline__ pft_dd dd_norm(double a, double b)
{
  const double s = a + b;
  return {s, b - (s - a)};
}
__host__ __device__ __forceinline__ pft_dd dd_mul(pft_dd a, pft_dd b)
{
  const double p = a.hi * b.hi;
  double e = fma(a.hi, b.hi, -p);
  e += a.hi * b.lo + a.lo * b.hi;
  return dd_norm(p, e);
}
// sign of x - m^(1/0.2) for the midpoint m = c + d (d = half the gap to a neighbour of c)
__host__ __device__ __forceinline__ int pow02_side(double x, double c, double d, double k)
{
  const pft_dd m = {c, d};
  const pft_dd m2 = dd_mul(m, m), m4 = dd_mul(m2, m2), m5 = dd_mul(m4, m);
  // T = m5 (1 - k): m5.hi - m5.hi k + m5.lo
  const double corr = -(m5.hi * k) + m5.lo;
  const double s = x - m5.hi;                 // exact when x and m5.hi are close (Sterbenz)
  const double r = s - corr;
  return r > 0.0 ? 1 : (r < 0.0 ? -1 : 0);
}
// c: a candidate within 1 ulp of x^0.2 (ocml's pow on the device)
__host__ __device__ __forceinline__ double pow02_fix(double x, double c)
{
  if (!(x > 0x1p-900 && x < 0x1p900) || !(c > 0.0 && c < 0x1p200)) return c;
  const double k = 25.0 * (0x1p-54 / 5.0) * log(c);
  const double up = nextafter(c, INFINITY), dn = nextafter(c, 0.0);
  if (pow02_side(x, c, 0.5 * (up - c), k) > 0) return up;
  if (pow02_side(x, c, 0.5 * (dn - c), k) < 0) return dn;
  return c;
}
__device__ __forceinline__ double pow02_rn(double x) { return pow02_fix(x, pow(x, 0.2)); }

// One thread: the step-size control of hybrid2.c:578-611 (rk_solver.c run_fused_impl restates it
// on the host) for the step (t, h) whose error norm bits epsb / non-finite flag nf were just
// reduced: the next step's (t, h) when it is accepted, a skip when it is rejected or hit a NaN.
// pow is the only operation not correctly rounded by IEEE: pow02_rn here, glibc on the host,
// which agree but for glibc's rare misrounded cases; the host takes its own decision and keeps
// the gated step only if both agree bit for bit (otherwise it discards it and launches the step
// again with its own h).
__device__ __forceinline__ void gate_decide(const StageArgs& a, double t, double h, unsigned long long epsb, int nf,
                                            bool have_eps)
{
  double eps = __longlong_as_double((long long)epsb);
  unsigned long long v = a.gdec_seq | PFT_GATE_SKIP, tb = 0, hb = 0;
  if (have_eps && !(a.d_nan && nf)) {                                      // :493-503
    const double h3 = h / 3.0;
    if (a.d_local) eps *= fabs(h3);                                        // :578
    const double new_h = ((eps > 0.0) ? pow02_rn((a.d_delta / eps)) * 0.8 : 2.0) * h;   // :580
    if (eps < a.d_delta || fabs(h) < a.d_hmin) {                           // :599-611
      const double tn = t + h;                                             // :652
      const double hn = (fabs(a.d_final - tn) <= fabs(new_h)) ? a.d_final - tn : new_h;   // :743-761
      tb = (unsigned long long)__double_as_longlong(tn);
      hb = (unsigned long long)__double_as_longlong(hn);
      if (a.d_flip > 0 && a.gdec_seq % (unsigned long long)a.d_flip == 0) hb ^= 1ULL;
      v = a.gdec_seq;
    }
  }
  a.gdev[1] = tb;
  a.gdev[2] = hb;
  __hip_atomic_store(a.gdev, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(a.gpin + 1, tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(a.gpin + 2, hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(a.gpin, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a value the error norm never takes (a NaN pattern: the max skips NaN) nor the flag
#define PFT_PUB_SENTINEL 0xFFF8DEADBEEF0001ULL

// The error norm's max over the workgroups of a launch (hybrid2.c:507-524 over the slab), and with
// it the count of finished workgroups whose last one publishes: arrivals on one address serialise
// at the memory side (~12 ns each), so a launch of ~500 short workgroups that all finish at once
// spent ~6 us in that queue (stage 5 at 100^3: 13.5 against 7 us for stage 4).  Workgroups
// arrive on one of PFT_EPS_SHARDS shards (blockIdx % shards: the dispatcher deals consecutive
// blocks to different XCDs) and the last of each shard forwards its shard's max to the launch's
// accumulator -- the same max, a tenth of the queue.  Every word is reset by the workgroup that
// reads it last, so the next launch on the stream finds them zero.
#define PFT_EPS_SHARDS 8
struct EpsShard {
  unsigned long long max;   // bit pattern of the shard's max (non-negative doubles order as their bits)
  unsigned int nf, cnt;     // non-finite flag, finished workgroups
  unsigned long long pad[6];  // one 64-byte line per shard
};

// called by one thread per workgroup after its block-level max bm / flag bnf; pub: the pinned host
// slot of an in-kernel publication (null: the accumulator is read after the launch)
__device__ __forceinline__ void eps_arrive(double bm, int bnf, EpsShard* shards, unsigned long long* eps_bits,
                                           unsigned int* nonfinite, unsigned long long* pub, unsigned int* pub_count)
{
  const unsigned nb = gridDim.x, b = blockIdx.x % PFT_EPS_SHARDS;
  const unsigned nsh = nb < PFT_EPS_SHARDS ? nb : PFT_EPS_SHARDS;             // shards with workgroups
  const unsigned in_shard = (nb - b + PFT_EPS_SHARDS - 1) / PFT_EPS_SHARDS;   // workgroups of shard b
  EpsShard* sh = shards + b;
  if (bm > 0.0) atomicMax(&sh->max, (unsigned long long)__double_as_longlong(bm));   // NaN never wins
  if (bnf) atomicOr(&sh->nf, 1u);
  // this workgroup's atomics are performed (memory-side) before it is counted
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (atomicAdd(&sh->cnt, 1u) != in_shard - 1) return;
  const unsigned long long m = atomicExch(&sh->max, 0ULL);
  const unsigned int f = atomicExch(&sh->nf, 0u);
  atomicExch(&sh->cnt, 0u);
  if (m) atomicMax(eps_bits, m);
  if (f) atomicOr(nonfinite, 1u);
  if (!pub) return;
  // the last shard to finish reads the final max, resets the accumulator and publishes both words
  // to the host, which polls them (no publish kernel, no event: pft_slab_eps_fetch)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (atomicAdd(pub_count, 1u) != nsh - 1) return;
  const unsigned long long e = atomicExch(eps_bits, 0ULL);
  const unsigned int ff = atomicExch(nonfinite, 0u);
  atomicExch(pub_count, 0u);
  __hip_atomic_store(pub, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(pub + 1, (unsigned long long)ff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Deferred publication (single slab / ipc, the speculative path): the error-norm launch does no
// atomics at all -- each workgroup stores its (max bits, non-finite flag) to part[2 b], part[2 b + 1]
// -- and the NEXT launch on the stream, the speculative stage 1, which follows it in every step,
// reduces them in one extra workgroup and publishes to the pinned host slot while its other
// workgroups compute.  The reduction leaves the error-norm launch's critical path (its last
// workgroups spent ~1-2 us in the arrival atomics), and the kernel boundary orders the plain stores
// before the reads.  One block of 256 threads; called with the block's threads.
__device__ __forceinline__ void eps_part_load(const unsigned long long* __restrict__ part, int n, unsigned long long& m,
                                              unsigned long long& f)
{
  m = 0;
  f = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const unsigned long long b = part[2 * i], nf = part[2 * i + 1];
    m = b > m ? b : m;   // non-negative doubles (and +0) order as their bit patterns
    f |= nf;
  }
}
__device__ __forceinline__ void eps_part_publish(unsigned long long m, unsigned long long f, unsigned long long* pub,
                                                 unsigned long long* mo = nullptr, unsigned long long* fo = nullptr)
{
  __shared__ unsigned long long rm[4], rf[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long om = __shfl_xor(m, off, 64), of = __shfl_xor(f, off, 64);
    m = om > m ? om : m;
    f |= of;
  }
  if ((threadIdx.x & 63) == 0) {
    rm[threadIdx.x >> 6] = m;
    rf[threadIdx.x >> 6] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      m = rm[w] > m ? rm[w] : m;
      f |= rf[w];
    }
    __hip_atomic_store(pub, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(pub + 1, f ? 1ULL : 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (mo) *mo = m;
    if (fo) *fo = f;
  }
}
__device__ __forceinline__ void eps_reduce_publish(const unsigned long long* __restrict__ part, int n,
                                                   unsigned long long* pub, unsigned long long* mo = nullptr,
                                                   unsigned long long* fo = nullptr)
{
  unsigned long long m, f;
  eps_part_load(part, n, m, f);
  eps_part_publish(m, f, pub, mo, fo);
}

// a workgroup's contribution in the deferred form
__device__ __forceinline__ void eps_store_part(unsigned long long* part, double bm, int bnf)
{
  part[2 * blockIdx.x] = bm > 0.0 ? (unsigned long long)__double_as_longlong(bm) : 0ULL;   // NaN never wins
  part[2 * blockIdx.x + 1] = bnf ? 1ULL : 0ULL;
}

__global__ __launch_bounds__(256) void eps_reduce_kernel(const unsigned long long* part, int n,
                                                         unsigned long long* pub)
{
  eps_reduce_publish(part, n, pub);
}


__device__ __forceinline__ int xcd_remap(int b, int n)
{
  // bijective: the blocks the dispatcher deals to one XCD (b % 8 equal) get consecutive ids
  const int q = n >> 3, r = n & 7, x = b & 7, l = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
}

template <int STAGE, bool GLS>
__device__ __forceinline__ double combine(const StageArgs& a, int q, long o, double K, double* m, bool& nf)
{
  // returns the value written to `out` (not used for stage 0)
  const double xv = a.x[q * a.fs + o];
  if (STAGE == 1) {
    a.kout[q * a.fs + o] = K;
    a.out[q * a.fs + o] = K * a.coef + xv;                               // hybrid2.c:388
  } else if (STAGE == 2) {
    const double k1 = a.k1[q * a.fs + o];
    a.out[q * a.fs + o] = (k1 + K) * a.coef + xv;                        // :408
  } else if (STAGE == 3) {
    const double k1 = a.k1[q * a.fs + o];
    a.kout[q * a.fs + o] = K;
    a.out[q * a.fs + o] = (k1 + 3.0 * K) * a.coef + xv;                  // :428
  } else if (STAGE == 4) {
    const double k1 = a.k1[q * a.fs + o], k3 = a.k3[q * a.fs + o];
    a.kout[q * a.fs + o] = K;
    a.out[q * a.fs + o] = (0.5 * k1 - 1.5 * k3 + 2.0 * K) * a.h + xv;   // :449
  } else if (STAGE == 5) {
    const double k1 = a.k1[q * a.fs + o], k3 = a.k3[q * a.fs + o], k4 = a.k4[q * a.fs + o];
    const double em = q == 0 ? a.em0 : (q == 1 ? a.em1 : a.em2);
    const double e = em * fabs(0.2 * k1 - 0.9 * k3 + 0.8 * k4 - 0.1 * K);   // :521
    if (e > *m) *m = e;                                                  // :522 (NaN never wins)
    nf |= !isfinite(e);
    a.out[q * a.fs + o] = xv + a.coef * (0.5 * (k1 + K) + 2.0 * k4);   // :667
  }
  return 0.0;
}

template <int STAGE, int MODE, bool GLS>
__global__ __launch_bounds__(PFT_BLOCK) void merson_stage(StageArgs a, pft_consts c)
{
  const int lin = xcd_remap(blockIdx.x, a.ntile * a.nchunk);
  const int tile = lin % a.ntile, chunk = lin / a.ntile;
  const int cell = tile * PFT_BLOCK + threadIdx.x;
  const bool active = cell < a.plane;
  const int cc = active ? cell : a.plane - 1;
  const int j = cc / a.n1, i = cc - j * a.n1;
  const int kb = a.k_begin + chunk * a.kz;
  const int ke = min(kb + a.kspan, a.k_end);

  // neighbour offsets within a plane, mirrored at the x/y walls (equation.c:137-161)
  const int oxm = i > 0 ? -1 : 0, oxp = i < a.n1 - 1 ? 1 : 0;
  const int oym = j > 0 ? -a.n1 : 0, oyp = j < a.n2 - 1 ? a.n1 : 0;

  const double* fin[3] = {a.in, a.in + a.fs, GLS ? a.x + 2 * a.fs : a.in + 2 * a.fs};

  double m = 0.0;
  bool nf = false;
  // software pipeline over the z-march (the loads of plane k+1's x/y neighbours and of plane
  // k+2's centre are in flight while plane k is computed):
  //   zm/zc/zp: centres of planes k-1, k, k+1;  nb: x/y neighbours of plane k;
  //   zn: centre of plane k+2 and nn: x/y neighbours of plane k+1 (prefetched)
  double zm[3], zc[3], zp[3], zn[3], nb[3][4], nn[3][4];
  if (kb < ke) {
    const long o0 = (long)(kb + 1) * a.plane + cc;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      zc[q] = fin[q][o0];
      // bottom wall: mirror (equation.c:164-174); slab interface: ghost plane
      zm[q] = (kb == 0 && !a.has_below) ? zc[q] : fin[q][o0 - a.plane];
      zp[q] = (kb == a.n3 - 1 && !a.has_above) ? zc[q] : fin[q][o0 + a.plane];
      nb[q][0] = fin[q][o0 + oxm];
      nb[q][1] = fin[q][o0 + oxp];
      nb[q][2] = fin[q][o0 + oym];
      nb[q][3] = fin[q][o0 + oyp];
    }
  }
  for (int k = kb; k < ke; ++k) {
    const long o = (long)(k + 1) * a.plane + cc;
    const bool top = (k == a.n3 - 1) && !a.has_above;
    // pointwise operands of this plane's stage combine, issued before the stencil arithmetic
    double xv[3], k1v[3], k3v[3], k4v[3];
    if (STAGE >= 1) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (GLS && q == 2) continue;
        xv[q] = a.x[q * a.fs + o];
        if (STAGE >= 2) k1v[q] = a.k1[q * a.fs + o];
        if (STAGE >= 4) k3v[q] = a.k3[q * a.fs + o];
        if (STAGE >= 5) k4v[q] = a.k4[q * a.fs + o];
      }
    }
    // prefetch for the next plane
    if (k + 1 < ke) {
      const long o1 = o + a.plane;
      const bool top2 = (k + 1 == a.n3 - 1) && !a.has_above;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        nn[q][0] = fin[q][o1 + oxm];
        nn[q][1] = fin[q][o1 + oxp];
        nn[q][2] = fin[q][o1 + oym];
        nn[q][3] = fin[q][o1 + oyp];
        zn[q] = top2 ? 0.0 : fin[q][o1 + a.plane];
      }
    }
    Col col[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      col[q].c = zc[q];
      col[q].xm = nb[q][0];
      col[q].xp = nb[q][1];
      col[q].ym = nb[q][2];
      col[q].yp = nb[q][3];
      col[q].zm = zm[q];
      col[q].zp = top ? zc[q] : zp[q];               // top wall: mirror ...
    }
    if (top) col[0].zp = a.T_top;                    // ... except Dirichlet u (equation.c:175-183)
    double du = 0.0, dp = 0.0;
    const double un = a.noise ? zc[0] + a.noise[(long)k * a.plane + cc] : zc[0];
    rhs_cell<MODE>(c, col[0], col[1], col[2], un, du, dp);
    if (active) {
      if (STAGE == 0) {
        a.kout[o] = du;
        a.kout[a.fs + o] = dp;
        a.kout[2 * a.fs + o] = 0.0;
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          if (GLS && q == 2) continue;
          const double K = q == 0 ? du : (q == 1 ? dp : 0.0);   // dgl = 0 (equation.c:731)
          const long e = q * a.fs + o;
          if (STAGE == 1) {
            a.kout[e] = K;
            a.out[e] = K * a.coef + xv[q];                                         // hybrid2.c:388
          } else if (STAGE == 2) {
            a.out[e] = (k1v[q] + K) * a.coef + xv[q];                              // :408
          } else if (STAGE == 3) {
            a.kout[e] = K;
            a.out[e] = (k1v[q] + 3.0 * K) * a.coef + xv[q];                        // :428
          } else if (STAGE == 4) {
            a.kout[e] = K;
            a.out[e] = (0.5 * k1v[q] - 1.5 * k3v[q] + 2.0 * K) * a.h + xv[q];     // :449
          } else if (STAGE == 5) {
            const double em = q == 0 ? a.em0 : (q == 1 ? a.em1 : a.em2);
            const double ev = em * fabs(0.2 * k1v[q] - 0.9 * k3v[q] + 0.8 * k4v[q] - 0.1 * K);  // :521
            if (ev > m) m = ev;                                                    // :522 NaN never wins
            nf |= !isfinite(ev);
            a.out[e] = xv[q] + a.coef * (0.5 * (k1v[q] + K) + 2.0 * k4v[q]);      // :667
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      zm[q] = zc[q];
      zc[q] = zp[q];
      zp[q] = zn[q];
#pragma unroll
      for (int d = 0; d < 4; ++d) nb[q][d] = nn[q][d];
    }
  }

  if (STAGE == 5) {
    // block max of the error norm (exact, order-independent), one atomic per block
    __shared__ double red[PFT_BLOCK / 64];
    __shared__ int rnf[PFT_BLOCK / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double o = __shfl_xor(m, off, 64);
      if (o > m) m = o;
    }
    const int anynf = __any(nf);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[w] = m;
      rnf[w] = anynf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double bm = red[0];
      int bnf = rnf[0];
      for (int k = 1; k < PFT_BLOCK / 64; ++k) {
        if (red[k] > bm) bm = red[k];
        bnf |= rnf[k];
      }
      // non-negative doubles order like their bit patterns
      if (bm > 0.0) atomicMax(a.eps_bits, (unsigned long long)__double_as_longlong(bm));
      if (bnf) atomicOr(a.nonfinite, 1u);
    }
  }
}

// ------------------------------------------------------------------------------------------
// the LDS-tiled fused stage kernel (n1 even): a 256-thread workgroup owns a TX x TY tile of the
// (x, y) plane, two x-adjacent cells per thread (16-byte loads and stores everywhere), and marches
// kz planes in z.  Plane k of the stage input sits in LDS with a halo (one row above/below, one
// 16-byte pair left/right), so each input value is fetched from memory once per plane instead
// of five times; plane k+1 is staged into the second LDS buffer while plane k is computed (the
// thread's own centre values double as the z+1 neighbours, the halo ring is one 16-byte load per
// thread).  The z-neighbours stay in registers.

typedef double dbl2 __attribute__((ext_vector_type(2)));

// LDS doubles per field and plane of merson_fused: (2 gwx + 4)(gty + 2) <= 680 (64 x 8 tiles)
#define PFT_FUSED_LF 680

// (non-temporal loads measured -25%, non-temporal stores +-0: plain accesses)
__device__ __forceinline__ dbl2 ld2(const double* p) { return *reinterpret_cast<const dbl2*>(p); }
__device__ __forceinline__ void st2(double* p, dbl2 v) { *reinterpret_cast<dbl2*>(p) = v; }

// ------------------------------------------------------------------------------------------
// the recompute kernel (default): an LDS tile, and no stage-input ("aux") array exists.
// The reference writes aux = combine(x, K...) after each stage and the next RHS reads it
// (hybrid2.c:378-450); here each stage kernel reads x and the K's its input is made of and
// evaluates the same combine, with the same operands in the same order, while staging the plane
// into LDS -- bit-identical inputs, and per cell-step 54 instead of 72 doubles of HBM traffic
// (SURVEY 8(d)'s "fused lower bound", 432 B).  Stage s writes only K_s (stage 5: x(t+h)).

struct Ops {             // operands of one 16-byte cell pair of one field
  dbl2 x, k1, k2, k3, k4;
};

template <int STAGE, bool GLS>
__device__ __forceinline__ void load_ops(const StageArgs& a, int q, long o, Ops& r)
{
  r.x = ld2(a.x + q * a.fs + o);
  if (GLS && q == 2) return;                     // dgl == 0: the gl input is x (F4)
  if (q == 2) {
    // gl's K's are the literal 0.0 the model's RHS writes for dgl (equation.c:731,874): never
    // stored, never loaded; the stage combines still run on them (stage_in, stage 5), so the gl
    // stage inputs and x(t+h) carry the reference's bits, signed zeros included
    constexpr dbl2 z = {0.0, 0.0};
    r.k1 = z; r.k2 = z; r.k3 = z; r.k4 = z;
    return;
  }
  if (STAGE >= 2 && STAGE != 3) r.k1 = ld2(a.k1 + q * a.fs + o);
  if (STAGE == 3) r.k2 = ld2(a.k2 + q * a.fs + o);   // S = K1 + K2, stored by stage 2
  if (STAGE >= 4) r.k3 = ld2(a.k3 + q * a.fs + o);
  if (STAGE == 5) r.k4 = ld2(a.k4 + q * a.fs + o);
}

template <int STAGE, bool GLS>
__device__ __forceinline__ dbl2 stage_in(const StageArgs& a, int q, const Ops& r)
{
  if (STAGE <= 1 || (GLS && q == 2)) return r.x;
  dbl2 v;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (STAGE == 2) v[s] = r.k1[s] * a.cin + r.x[s];                                      // hybrid2.c:388
    if (STAGE == 3) v[s] = r.k2[s] * a.cin + r.x[s];                                      // :408 (S = K1 + K2)
    if (STAGE == 4) v[s] = (r.k1[s] + 3.0 * r.k3[s]) * a.cin + r.x[s];                    // :428
    if (STAGE == 5) v[s] = (0.5 * r.k1[s] - 1.5 * r.k3[s] + 2.0 * r.k4[s]) * a.cin + r.x[s];  // :449
  }
  return v;
}

template <bool GLS>
__device__ __forceinline__ void keep5(int q, const Ops& r, dbl2& x, dbl2& k1, dbl2& k4, dbl2& E)
{
  x = r.x;
  if (q == 2) return;
  k1 = r.k1;
  k4 = r.k4;
#pragma unroll
  for (int s = 0; s < 2; ++s) E[s] = 0.2 * r.k1[s] - 0.9 * r.k3[s] + 0.8 * r.k4[s];   // hybrid2.c:521 prefix
}

template <int STAGE, int MODE, bool GLS>
__global__ __launch_bounds__(PFT_FBLOCK) __attribute__((amdgpu_waves_per_eu(STAGE >= 1 ? 2 : 3))) void merson_fused(StageArgs a, pft_consts c)
{
  // tile geometry chosen by the host per grid (fused_geometry): gwx pairs x gty rows, so that the
  // tiles fit n1 and n2 without mostly-idle edge workgroups (n1 = 200: 50 x 10 cells)
  const int WX = a.gwx, TY = a.gty, TX = 2 * WX, LW = TX + 4, LH = TY + 2, NH = LW + 2 * TY;
  __shared__ __attribute__((aligned(16))) double lds[2][3][PFT_FUSED_LF];

  // A gated launch runs iff the step it belongs to was accepted, on the decided (t, h) (gate words
  // [0] sequence, [1] t, [2] h).  The words are loaded here, beside the prologue's operand loads
  // (which need no scalar of the step), and checked after them: one memory round trip before the
  // stencil instead of two dependent ones (the check and then t, h) ahead of it.
  unsigned long long gw0 = 0, gw1 = 0, gw2 = 0;
  if (a.gate) {
    gw0 = __hip_atomic_load(a.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gw1 = a.gate[1];
    gw2 = a.gate[2];
  }
  if (STAGE == 1 && (a.npart > 0 || a.gdev) && (int)blockIdx.x == a.nbw + a.nint) {
    // the extra workgroup of a speculative stage 1: the previous launch's error norm, then (gated
    // steps) the decision on the step it ended
    unsigned long long m = 0, f = 0;
    if (a.npart > 0) eps_part_load(a.part, a.npart, m, f);
    if (a.gate) {
      if (gw0 != a.gseq) return;       // (uniform: every thread read the same word)
      a.dt = __longlong_as_double((long long)gw1);
      a.dh = __longlong_as_double((long long)gw2);
    }
    if (a.npart > 0) eps_part_publish(m, f, a.pub, &m, &f);
    if (a.gdev && threadIdx.x == 0) gate_decide(a, a.dt, a.dh, m, (int)f, a.npart > 0);
    return;
  }
  const int ntx = (a.n1 + TX - 1) / TX;
  // inline boundary: the leading workgroups (dispatched first) produce the planes the exchange sends
  const bool bw = (int)blockIdx.x < a.nbw;
  const int lin = bw ? xcd_remap(blockIdx.x, a.nbw) : xcd_remap(blockIdx.x - a.nbw, a.nint);
  const int tile = lin % a.ntile, cq = lin / a.ntile;
  const int chunk = bw ? (a.bends ? (cq ? a.nchunk - 1 : 0) : cq) : a.c0 + cq;
  const bool bshort = bw && !a.bends;
  const int x0 = (tile % ntx) * TX, y0 = (tile / ntx) * TY;
  // threads beyond the WX x TY tile (256 > WX * TY) shadow the tile's last thread: the same loads
  // and LDS writes (same values to the same slots), no global stores
  const int tt = min((int)threadIdx.x, WX * TY - 1);
  const int tx = tt % WX, ty = tt / WX;
  const int i0 = x0 + 2 * tx, j = y0 + ty;
  const bool active = (i0 < a.n1) && (j < a.n2) && (int)threadIdx.x < WX * TY;
  const long po = (long)(j < a.n2 ? j : a.n2 - 1) * a.n1 + (i0 < a.n1 ? i0 : a.n1 - 2);
  const int kb = bshort ? chunk * (a.n3 - 2) : a.k_begin + chunk * a.kz;
  const int ke = bshort ? kb + 2 : min(kb + a.kspan, a.k_end);
  const int lo = (ty + 1) * LW + 2 + 2 * tx;

  const int t = threadIdx.x;
  const bool hact = t < 3 * NH;
  const int hf = hact ? t / NH : 0, h = hact ? t % NH : 0;
  int hr, hcp;
  if (h < LW / 2) { hr = 0; hcp = h; }
  else if (h < LW) { hr = LH - 1; hcp = h - LW / 2; }
  else { const int q = h - LW; hr = 1 + q / 2; hcp = (q & 1) ? LW / 2 - 1 : 0; }
  const int hi = x0 - 2 + 2 * hcp, hj = y0 + hr - 1;
  // Walls in LDS: a halo pair outside the domain holds the mirror image the reference's ghost
  // fill puts there (equation.c:137-174: ghost -1-m = interior m), so the stencil reads its x/y
  // neighbours without selects.  Pair (-2,-1) = (v1, v0): pair (0,1) swapped; pair (n1, n1+1) =
  // (v[n1-1], v[n1-2]): pair (n1-2, n1-1) swapped (held in natural order, below); rows -1 / n2 =
  // rows 0 / n2-1.
  const long hp = (long)(hj < 0 ? 0 : (hj >= a.n2 ? a.n2 - 1 : hj)) * a.n1 +
                  (hi < 0 ? 0 : (hi >= a.n1 ? a.n1 - 2 : hi));
  const int hl = hr * LW + 2 * hcp;
  // An inactive pair just right of the domain (partial tile) is the mirror of the last pair.  Every
  // pair, mirrored ones included, is stored in natural order (16-byte stores), and the thread next
  // to a mirrored pair reads its other cell instead: (-2, -1) holds (v0, v1), cell -1 = its even
  // cell; (n1, n1 + 1) holds (v[n1-2], v[n1-1]), cell n1 = its odd cell (xma / xpa: offsets of the
  // x-neighbour reads).  (Round 3 stored mirrored pairs as two 8-byte halves at exchanged offsets:
  // 2-way LDS bank conflicts)
  const int xma = i0 - 2 < 0 ? 1 : 0, xpa = i0 + 2 >= a.n1 ? 1 : 0;

  double m = 0.0;
  bool nf = false;
  dbl2 zm[3], zc[3], zp[3];
  constexpr bool FLUX = MODE != 10 && MODE != 11;
  // face reuse (rhs_cell_f) in every stage; stage 5 holds two planes of combine operands beside
  // the z-face carry (235 VGPRs, no spills)
  // two-deep z pipeline (stages 1-4): the raw operands of plane k+2 are loaded while plane k is
  // computed (the stage input of plane k+1 is its z+1 neighbour, so a one-deep pipeline waits for
  // its loads before the stencil).  It costs the operand registers: 2 waves/SIMD.  Measured at
  // 400^3: stages 3-4 0.258 vs 0.288-0.296 ms, stage 1 0.158 vs 0.166, stage 2 0.217 vs 0.222.
  constexpr bool DEEP = STAGE >= 1 && STAGE <= 4;
  Ops pn[3], ph;                       // DEEP: operands of plane k+1 (centre, halo pair)
  FaceT fz[2];                         // z-face below plane k of each cell of the pair
  // stage 2 stores S = K1 + K2 (stage 3's input combine, hybrid2.c:408), K1 carried in registers
  // (re-loading it one plane later measured 4% slower)
  constexpr bool SUM2 = STAGE == 2;
  dbl2 s2c[3], s2n[3];                 // SUM2: K1 of planes k and k+1 (the stored sum's operand)
  // stage 5 keeps x, K1, K4 and the K1/K3/K4 part of the error norm of planes k and k+1
  // (re-loading them one plane later misses the 4 MiB L2: 0.52 vs 0.65 ms at 400^3)
  dbl2 cx[3], ck1[3], ck4[3], cE[3], nx[3], nk1[3], nk4[3], nE[3];
  int cur = 0;
  const long o0 = (long)(kb + 1) * a.plane + po;
  const bool wlo = kb == 0 && !a.has_below;
  const long ob = wlo ? o0 : o0 - a.plane;
  Ops cop[3], bop[3], hop;
  if (kb < ke) {
#pragma unroll
    for (int q = 0; q < 3; ++q) load_ops<STAGE, GLS>(a, q, o0, cop[q]);
#pragma unroll
    for (int q = 0; q < 3; ++q) load_ops<STAGE, GLS>(a, q, ob, bop[q]);
    load_ops<STAGE, GLS>(a, hf, (long)(kb + 1) * a.plane + hp, hop);
  }
  if (a.gate) {
    if (gw0 != a.gseq) return;         // rejected (or NaN): leave before any store
    const double gt = __longlong_as_double((long long)gw1), gh = __longlong_as_double((long long)gw2);
    gate_scalars<STAGE>(a, c, gt, gh);
    a.dt = gt;
    a.dh = gh;
  }
  if (kb < ke) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      zc[q] = stage_in<STAGE, GLS>(a, q, cop[q]);
      if constexpr (SUM2) s2c[q] = cop[q].k1;
      if (STAGE == 5) keep5<GLS>(q, cop[q], cx[q], ck1[q], ck4[q], cE[q]);
      zm[q] = wlo ? zc[q] : stage_in<STAGE, GLS>(a, q, bop[q]);
      st2(&lds[0][q][lo], zc[q]);
    }
    if (hact) st2(&lds[0][hf][hl], stage_in<STAGE, GLS>(a, hf, hop));
    // the DEEP look-ahead after those loads are consumed, as before: the loop then starts with
    // only the look-ahead in flight (with it issued together with the rest, the compiler's wait
    // placement serialised the loop's own look-ahead: stage 1 at 400^3 0.149 -> 0.175 ms)
    if constexpr (DEEP) {
      if (!((kb == a.n3 - 1) && !a.has_above)) {
#pragma unroll
        for (int q = 0; q < 3; ++q) load_ops<STAGE, GLS>(a, q, o0 + a.plane, pn[q]);
      }
      if (hact && kb + 1 < ke) load_ops<STAGE, GLS>(a, hf, (long)(kb + 2) * a.plane + hp, ph);
    }
    // the z-face below the chunk's first plane; later planes inherit it from the plane below
#pragma unroll
    for (int s = 0; s < 2; ++s)
      fz[s] = face_of(c, zm[1][s], zm[2][s], zm[0][s], zc[1][s], zc[2][s], zc[0][s], FLUX);
    __syncthreads();
  }
  for (int k = kb; k < ke; ++k) {
    const long o = (long)(k + 1) * a.plane + po;
    const bool top = (k == a.n3 - 1) && !a.has_above;
    const bool more = k + 1 < ke;
    // z+1 neighbours: the stage input of plane k+1 (interior, or the exchanged ghost plane)
    if (!top) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if constexpr (DEEP) {
          zp[q] = stage_in<STAGE, GLS>(a, q, pn[q]);
          if constexpr (SUM2) s2n[q] = pn[q].k1;
        } else {
          Ops nop;
          load_ops<STAGE, GLS>(a, q, o + a.plane, nop);
          zp[q] = stage_in<STAGE, GLS>(a, q, nop);
          if constexpr (SUM2) s2n[q] = nop.k1;
          if (STAGE == 5) keep5<GLS>(q, nop, nx[q], nk1[q], nk4[q], nE[q]);
        }
      }
    }
    dbl2 hv = {0.0, 0.0};
    if (more) {
#pragma unroll
      for (int q = 0; q < 3; ++q) st2(&lds[cur ^ 1][q][lo], zp[q]);
      if (hact) {
        if constexpr (DEEP) {
          hv = stage_in<STAGE, GLS>(a, hf, ph);
        } else {
          Ops tmp;
          load_ops<STAGE, GLS>(a, hf, (long)(k + 2) * a.plane + hp, tmp);
          hv = stage_in<STAGE, GLS>(a, hf, tmp);
        }
      }
    }
    if constexpr (DEEP) {
      // operands of plane k+2 (and its halo pair), in flight during the stencil of plane k
      if (more) {
        if (!((k + 1 == a.n3 - 1) && !a.has_above)) {
#pragma unroll
          for (int q = 0; q < 3; ++q) load_ops<STAGE, GLS>(a, q, o + 2 * a.plane, pn[q]);
        }
        if (hact && k + 2 < ke) load_ops<STAGE, GLS>(a, hf, (long)(k + 3) * a.plane + hp, ph);
      }
    }
    if (top) {                         // top wall (uniform): mirror p, gl; Dirichlet u (equation.c:175-183)
#pragma unroll
      for (int q = 1; q < 3; ++q) zp[q] = zc[q];
      zp[0] = dbl2{a.T_top, a.T_top};
    }
    double du[2], dp[2];
    FaceT fx;                          // the x-face between the pair's two cells
    // the y neighbours of both cells as one 16-byte LDS read per neighbouring pair (consecutive
    // lanes: no bank conflicts, where two 8-byte reads at a 16-byte lane stride conflict 2-way)
    dbl2 ym2[3], yp2[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      ym2[q] = ld2(&lds[cur][q][lo - LW]);
      yp2[q] = ld2(&lds[cur][q][lo + LW]);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Col col[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const double* L = lds[cur][q];
        const double cen = zc[q][s];
        col[q].c = cen;
        // x/y neighbours straight from LDS: the walls' mirror values are in the halo
        col[q].xm = s == 0 ? L[lo - 1 - xma] : zc[q][0];
        col[q].xp = s == 0 ? zc[q][1] : L[lo + 2 + xpa];
        col[q].ym = ym2[q][s];
        col[q].yp = yp2[q][s];
        col[q].zm = zm[q][s];
        col[q].zp = zp[q][s];
      }
      const double un = a.noise ? zc[0][s] + a.noise[(long)k * a.plane + po + s] : zc[0][s];
      const FaceT fxm =
          s == 0 ? face_of(c, col[1].xm, col[2].xm, col[0].xm, col[1].c, col[2].c, col[0].c, FLUX) : fx;
      FaceT fzp;
      rhs_cell_f<MODE>(c, col[0], col[1], col[2], un, fxm, fz[s], fx, fzp, du[s], dp[s]);
      fz[s] = fzp;
    }
    if (more && hact) st2(&lds[cur ^ 1][hf][hl], hv);
    if (active) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q == 2 && STAGE != 0 && (GLS || STAGE <= 4)) continue;   // gl's K's: literal zeros, never stored
        const dbl2 K = q == 0 ? dbl2{du[0], du[1]} : (q == 1 ? dbl2{dp[0], dp[1]} : dbl2{0.0, 0.0});
        const long e = q * a.fs + o;
        if (SUM2) {
          dbl2 S;
          const dbl2 k1c = s2c[q];
#pragma unroll
          for (int s = 0; s < 2; ++s) S[s] = k1c[s] + K[s];   // K1 + K2, hybrid2.c:408
          st2(a.kout + e, S);
        } else if (STAGE <= 4) {
          st2(a.kout + e, K);
        } else {
          // the combine operands of plane k, kept in registers since they were loaded
          // gl (q = 2): K1, K4 and the K part of the error norm are the literal zeros of dgl
          // (equation.c:731), so they are not carried in registers
          constexpr dbl2 zero2 = {0.0, 0.0};
          const bool z2 = q == 2;
          const dbl2 ox = cx[q], ok1 = z2 ? zero2 : ck1[q], ok4 = z2 ? zero2 : ck4[q];
          dbl2 oE = cE[q];
          if (z2) {
#pragma unroll
            for (int s = 0; s < 2; ++s) oE[s] = 0.2 * 0.0 - 0.9 * 0.0 + 0.8 * 0.0;   // :521 prefix
          }
          dbl2 r;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const double em = q == 0 ? a.em0 : (q == 1 ? a.em1 : a.em2);
            const double ev = em * fabs(oE[s] - 0.1 * K[s]);                                    // :521
            if (ev > m) m = ev;                                                               // NaN never wins
            nf |= !isfinite(ev);
            r[s] = ox[s] + a.coef * (0.5 * (ok1[s] + K[s]) + 2.0 * ok4[s]);                  // :667
          }
          if (!(q == 2 && a.gl_keep)) st2(a.out + e, r);
        }
      }
    }
    __syncthreads();
    cur ^= 1;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      zm[q] = zc[q];
      zc[q] = zp[q];
      if constexpr (SUM2) s2c[q] = s2n[q];
      if (STAGE == 5) { cx[q] = nx[q]; ck1[q] = nk1[q]; ck4[q] = nk4[q]; cE[q] = nE[q]; }
    }
  }

  if (STAGE == 5) {
    __shared__ double red[PFT_FBLOCK / 64];
    __shared__ int rnf[PFT_FBLOCK / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(m, off, 64);
      if (ov > m) m = ov;
    }
    const int anynf = __any(nf);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[w] = m;
      rnf[w] = anynf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double bm = red[0];
      int bnf = rnf[0];
      for (int q = 1; q < PFT_FBLOCK / 64; ++q) {
        if (red[q] > bm) bm = red[q];
        bnf |= rnf[q];
      }
      if (a.part) eps_store_part(a.part, bm, bnf);
      else eps_arrive(bm, bnf, a.shards, a.eps_bits, a.nonfinite, a.pub, a.pub_count);
    }
  }
  if (bw) {
    // an inline boundary workgroup (as merson_pair's): stores done, L2 written back, counted.  (A
    // gated launch, which may leave before its stores, never runs inline: run_stage)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_fetch_add(a.bdone, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------------------------------
// the pair kernel: two consecutive Merson stages (2+3, or 4+5) in ONE z-march.
//
// Stage B's input at a cell is a pointwise combine of x, the K's and stage A's K there
// (hybrid2.c:408 / :449), so stage B's 7-point stencil at the tile needs stage A's K on the tile
// plus a one-cell ring, and stage A's stencil there needs stage A's input on a two-cell ring.  A
// workgroup recomputes stage A on its ring (the neighbouring workgroups compute the same cells
// with the same operands in the same order: the same bits) and never stores it: K2 and K4 do
// not exist in HBM, and neither stage re-reads x and the K's the other one read.  Per cell-step:
//   stages 2, 3 apart: (5 + 2) + (5 + 2) = 14 doubles -> pair 2+3: x, K1 in, K3 out = 7
//   stages 4, 5 apart: (7 + 2) + (9 + 2) = 20 doubles -> pair 4+5: x, K1, K3 in, x(t+h) out = 9
// so the step (speculative stage 1 + the two pairs) moves 21 instead of 39 doubles per cell.
//
// Workgroup (PFT_PBLOCK threads): an R0 tile of tx x ty cells (tx even) is stage B's output.
// Thread (px, py) holds the cell pair (x0 - 2 + 2 px, x0 - 1 + 2 px) of row y0 - 2 + py, for px
// in [0, tx/2 + 2) and py in [0, ty + 4): the tile plus a two-cell ring (R2).  Every thread loads
// its pair's operands and writes stage A's input into LDS (plane ring lA); threads of rows
// 1..ty+2 (the tile plus a one-cell ring, R1) evaluate stage A at their pair and write stage B's
// input into LDS (plane ring lB); threads of the tile evaluate stage B.  A position outside the
// domain (walls) holds the mirror image the reference's ghost fill puts there (equation.c:137-174:
// ghost -1-m = interior m): its thread loads the mirrored in-domain pair ("acting" pair), stores
// it into LDS with its halves exchanged when mirrored in x, and evaluates stage A exactly as the
// acting pair's own thread does -- so the mirrored stage-B input is the reference's bit for bit.
// z neighbours of both levels are read from the plane rings (own pair: written by the thread
// itself; x/y neighbours: written one iteration earlier, behind the barrier).
//
// Positions beyond the 512 threads (round 6, the 40 x 20 tile: 22 x 24 = 528 positions).  The
// last ring row (py = ty + 3) is only read, as the y neighbours of stage A's last row; its
// positions past thread 511 (at most PFT_PAIR_NEX, all in that row) are loaded by lanes 0..15 of
// the last wave as LDS DMA (global_load_lds_dwordx4: no registers -- the kernel has none to spare
// at 256 VGPRs) into the staging array lX one plane ahead, and at the next iteration's start the
// same lanes combine them into stage A's input and store it into lA with the other positions'.
// The taller tile evaluates stage B on 400 positions instead of 380 with the same wave-phases per
// plane, n2 = 200 / 400 is cut into 10 / 20 tile rows with no idle row (19-row tiles: 11 / 22, the
// last one half empty), and 400^3 runs its 50 tiles x 5 z-chunks in one round of 250 workgroups
// (55 x 9 in two rounds before): DESIGN.md section 8.0.
#define PFT_PBLOCK 512
#define PFT_PAIR_NEX 16
// LDS layout of a field plane: the positions' cell pairs side by side (16 bytes a slot, PairLds
// below), position (px, py) at slot PFT_PAIR_PADP + py LWP + px.  (The layout with the even and
// odd cells in two halves, conflict-free 8-byte accesses, was removed in round 5: PairLds.)
#define PFT_PAIR_PADP 2         // slots before / after the positions of each half: the discarded
                                // outer cell of a ring pair reads one slot beyond its row
#define PFT_PAIR_H 532          // pair slots of a stage-A field plane (rows 0..ty+3 at the row pitch)
#define PFT_PAIR_HB 488         // slots of a stage-B plane in the interleaved layout (rows 1..ty+2)
// The row pitch LWP (pairs) is a template parameter, a compile-time constant so that every LDS
// access is a per-lane base + an immediate offset: 22 (tiles up to 40 cells wide, 20 rows) or 12
// (up to 20 cells wide, 38 rows: n1 = 100 in 5 tiles of 20 where 40-wide tiles leave a sixth idle)
// measured crossover (profiles/r05_pair_threshold.txt, stage launches against pair kernels forced):
// 128^3 (2048 cells per CU) -10%, 136^3 (2456) -1.4%, 144^3 (2916) +16%, 152^3 (3429) +18%, 160^3
// (4000) +9%, 200^3 (7.8 Ki) +7-9%
#define PFT_PAIR_MIN_CELLS_PER_CU 2560

struct PairArgs {
  const double* x;
  const double* k1;
  const double* k3;     // pair 4+5 only
  double* out;          // pair 2+3: K3 (u, p); pair 4+5: x(t+h) (u, p; gl unless gl_keep)
  const double* noise;  // u_noise [k][j][i] or null
  unsigned long long* eps_bits;
  unsigned int* nonfinite;
  unsigned long long* pub;   // in-kernel publication of the error norm (as merson_fused<5>)
  unsigned int* pub_count;
  EpsShard* shards;    // the error norm's per-shard accumulators (eps_arrive)
  unsigned long long* part;   // deferred publication: this launch's workgroup partials (eps_store_part)
  long fs;
  int n1, n2, n3, plane;
  int has_below, has_above;   // z-neighbours: stage A also runs on the ghost plane next to each,
                              // from the two-plane halo (ghost + far ghost planes, pft_slab_far)
  int k_begin, k_end, kz, ntile, nchunk, ntx;
  int kspan;            // planes a chunk runs from its start (kz; 2 for the two-plane boundary launch)
  // inline boundary (PFT_K_INLINE, PFT_K_ENDS_FIRST): the grid's first nbw workgroups produce the
  // planes the exchange sends, each adding one to *bdone once they are written back (nbw 0: none).
  // bends 0: they run the two planes at each end (chunk 0: planes 0, 1; chunk 1: n3 - 2, n3 - 1)
  // and the other nint workgroups the chunks of [k_begin, k_end); bends 1: one launch of the whole
  // slab's chunks, the first and the last chunk of every tile column first, then chunks c0 ..
  int nbw, bends, c0, nint;
  unsigned long long* bdone;
  int tx, ty;           // R0 tile: tx cells (even) x ty rows
  double T_topA, T_topB;   // Dirichlet u above the top plane at the two stage times
  double cinA, cinB;    // stage-input coefficients: h/3, h/6 (2+3); h/8, h (4+5)
  double coef;          // x(t+h) coefficient h/3 (4+5)
  double em0, em1;
  // gl's K's are the literal zeros of dgl (equation.c:731,874), so every gl term of the step is a
  // per-launch constant the host evaluates with the reference's expression (pair_gl_consts):
  // stage A's and stage B's gl input are glA + x and glB + x, x(t+h) of gl is x + glX, and gl's
  // error-norm term is evgl.  GLX kernels (gl_static, or gl_keep: x's gl holds no -0.0 or NaN and
  // the coefficients are finite) read gl's inputs straight from x: glA + x == x bit for bit there.
  double glA, glB, glX, evgl;
  int gl_keep;
};
// byte offset of the kernel's second argument (pft_consts) in the kernarg segment
static constexpr unsigned PFT_PAIR_COFF =
    (unsigned)((sizeof(PairArgs) + alignof(pft_consts) - 1) / alignof(pft_consts) * alignof(pft_consts));

// The z-loop re-reads the kernel arguments (PairArgs, pft_consts) from the kernarg segment with
// scalar loads at each of its three phases (PFT_PAIR_BIND: the pointer is laundered through an
// empty asm, so the loads cannot be hoisted out of the loop).  Kept live across the whole loop,
// the ~25 model constants, the array bases and the step coefficients needed ~190 SGPRs: ~90 were
// spilled into VGPR lanes and re-read by ~160 v_readlane per iteration (pair 4+5 0.519 -> 0.486 ms
// at 400^3; pair 2+3 0.408 -> 0.403 ms).
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) char* pft_kptr;
#define PFT_PAIR_BIND(A, C)                                                                  \
  pft_kptr kq_##A = kbase;                                                                  \
  asm volatile("" : "+s"(kq_##A));                                                          \
  const PairArgs& A = *(const __attribute__((address_space(4))) PairArgs*)kq_##A;           \
  const pft_consts& C = *(const __attribute__((address_space(4))) pft_consts*)(kq_##A + PFT_PAIR_COFF)
#else
#define PFT_PAIR_BIND(A, C) \
  const PairArgs& A = a;    \
  const pft_consts& C = c
#endif

// operands of one cell pair: x (u, p, gl), K1 and K3 (u, p; gl's K's are the literal zeros of
// dgl, equation.c:731,874)
struct PairRaw {
  dbl2 x[3], k1[2], k3[2];
};

// 16-byte load / store at a byte offset from a wave-uniform base: the base stays in SGPRs and the
// per-lane offset is one 32-bit VGPR for every array (global_load saddr + voffset), instead of a
// 64-bit address per array and plane (pft_slab_pair_ok: a field is < 4 GiB)
__device__ __forceinline__ dbl2 ldb(const double* base, unsigned bo)
{
  return *reinterpret_cast<const dbl2*>(reinterpret_cast<const char*>(base) + bo);
}
__device__ __forceinline__ void stb(double* base, unsigned bo, dbl2 v)
{
  *reinterpret_cast<dbl2*>(reinterpret_cast<char*>(base) + bo) = v;
}

// operands of plane m in [-2, n3 + 1] (interior 0..n3-1; -1 and n3 the ghost planes, -2 and n3+1
// the far ghost planes of the two-plane halo) at byte offset bo = pbo(m).  The PairArgs pointers
// are the buffers' pointers minus one plane (run_pair): field q holds plane m at q fs + (m + 2)
// plane from there, so every offset is unsigned.  gl's x is loaded only where an input needs it.
template <int SA, bool GL = true>
__device__ __forceinline__ void pair_load(const PairArgs& a, unsigned bo, PairRaw& r)
{
#pragma unroll
  for (int q = 0; q < (GL ? 3 : 2); ++q) r.x[q] = ldb(a.x + q * a.fs, bo);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    r.k1[q] = ldb(a.k1 + q * a.fs, bo);
    if (SA == 4) r.k3[q] = ldb(a.k3 + q * a.fs, bo);
  }
}

// stage A's input (stage 2: hybrid2.c:388; stage 4: :428) -- the expressions of stage_in; gl:
// glA + x (the combine of its literal-zero K's, a per-launch constant), x itself under GLX
template <int SA, bool GLX>
__device__ __forceinline__ dbl2 pair_in_A(const PairArgs& a, int q, const PairRaw& r)
{
  if (q == 2) {
    if (GLX) return r.x[2];
    return dbl2{a.glA + r.x[2][0], a.glA + r.x[2][1]};
  }
  const dbl2 k1 = r.k1[q < 2 ? q : 0];
  const dbl2 k3 = r.k3[q < 2 ? q : 0];
  dbl2 v;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (SA == 2) v[s] = k1[s] * a.cinA + r.x[q][s];
    else v[s] = (k1[s] + 3.0 * k3[s]) * a.cinA + r.x[q][s];
  }
  return v;
}

// stage B's input from the operands and stage A's K at the cell (stage 3: (K1 + K2) h/6 + x,
// hybrid2.c:408; stage 5: (0.5 K1 - 1.5 K3 + 2 K4) h + x, :449)
template <int SA, bool GLX>
__device__ __forceinline__ dbl2 pair_in_B(const PairArgs& a, int q, const PairRaw& r, dbl2 KA)
{
  if (q == 2) {
    if (GLX) return r.x[2];
    return dbl2{a.glB + r.x[2][0], a.glB + r.x[2][1]};
  }
  const dbl2 k1 = r.k1[q < 2 ? q : 0];
  const dbl2 k3 = r.k3[q < 2 ? q : 0];
  dbl2 v;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (SA == 2) v[s] = (k1[s] + KA[s]) * a.cinB + r.x[q][s];
    else v[s] = (0.5 * k1[s] - 1.5 * k3[s] + 2.0 * KA[s]) * a.cinB + r.x[q][s];
  }
  return v;
}

// A field plane of a ring holds the positions' cell pairs side by side (slot p: doubles 2p, 2p + 1),
// mirrored positions in natural order (the neighbour reading one takes its other cell).  A cell read
// on its own is an 8-byte access at a 16-byte lane stride (2-way bank conflicts), so pair_rhs reads
// the y neighbours of both cells as one 16-byte access per neighbouring pair (consecutive lanes,
// conflict-free).  Measured against it and removed (A/B on one box each, 400^3;
// profiles/r04b_ab_small_grids_and_layouts.txt): the even and odd cells in two
// halves (every access conflict-free, no 16-byte accesses, more address registers): pair 2+3
// 0.357-0.359 ms against 0.352-0.356, pair 4+5 0.416-0.424 against 0.409-0.411 (a spill); the y
// neighbours as two 8-byte reads: pair 2+3 0.362-0.365, pair 4+5 0.410-0.415.
#define PFT_PAIR_OPN 400      // stage-B positions of a tile ((tx/2) ty, at most 400: pair_geometry_ok)
struct PairLds {
  __device__ static __forceinline__ dbl2 ld(const double* L, int p) { return ld2(L + 2 * p); }
  __device__ static __forceinline__ void st(double* L, int p, dbl2 v) { st2(L + 2 * p, v); }
  __device__ static __forceinline__ double cell(const double* L, int p, int s) { return L[2 * p + s]; }
};

// One 16-byte LDS DMA per active lane (global_load_lds_dwordx4): lane l of the wave writes the 16
// bytes at g into LDS byte address lds + 16 l.  Inline asm rather than
// __builtin_amdgcn_global_load_lds: hipcc treats the builtin's pending LDS write as a reason to wait
// for vmcnt(0) at the next barrier and at the next use of an ordinary load -- it would drain the
// look-ahead loads and the output stores every plane (MI355X guide, "Pipelining across barriers").
// Invisible to the compiler, the DMA is ordered by hand: its reader waits with a counted vmcnt
// (pair_x_wait), and the "memory" clobber keeps the reads of the previous plane's staging before it
// and the look-ahead loads after it.  M0 is not used by any other instruction of these kernels.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lds_dma16(unsigned lds, const void* base, unsigned off)
{
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(off), "s"(base) : "memory", "m0");
}
#pragma clang diagnostic pop
// the staging of the previous plane's DMA has landed: every vector-memory operation but the N
// youngest is done (loads, stores and LDS DMA count together in issue order, MI355X guide)
template <int N>
__device__ __forceinline__ void pair_x_wait()
{
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// the RHS of one cell pair (du, dp of both cells): centre zc, z neighbours zm / zp, x/y
// neighbours from the LDS field planes L[q] around slot p (even / odd halves, row pitch LWP); the
// x-face between the pair's cells is evaluated once and the z-face below is carried in fz
// (rhs_cell_f, bit-exact), as in merson_fused
template <int MODE, int LWP>
__device__ __forceinline__ void pair_rhs(const pft_consts& c, const double* L0, const double* L1, const double* L2,
                                         int p, int xmc, int xpc, const dbl2* zm, const dbl2* zc, const dbl2* zp,
                                         const double* nz, FaceT* fz, double* du, double* dp)
{
  constexpr bool FLUX = MODE != 10 && MODE != 11;
  using LD = PairLds;
  const double* L[3] = {L0, L1, L2};
  // the y neighbours of both cells as one 16-byte read per neighbouring pair (consecutive lanes,
  // conflict-free) instead of two 8-byte reads at a 16-byte lane stride
  dbl2 ym2[3], yp2[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    ym2[q] = LD::ld(L[q], p - LWP);
    yp2[q] = LD::ld(L[q], p + LWP);
  }
  FaceT fx;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    Col col[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const double cen = zc[q][s];
      col[q].c = cen;
      // the cell of the pair to the left / right next to this pair: its odd / even cell, or the
      // other one where that slot holds a mirrored position in natural order (xmc / xpc)
      col[q].xm = s == 0 ? LD::cell(L[q], p - 1, xmc) : zc[q][0];
      col[q].xp = s == 0 ? zc[q][1] : LD::cell(L[q], p + 1, xpc);
      col[q].ym = ym2[q][s];
      col[q].yp = yp2[q][s];
      col[q].zm = zm[q][s];
      col[q].zp = zp[q][s];
    }
    const double un = nz ? zc[0][s] + nz[s] : zc[0][s];
    const FaceT fxm =
        s == 0 ? face_of(c, col[1].xm, col[2].xm, col[0].xm, col[1].c, col[2].c, col[0].c, FLUX) : fx;
    FaceT fzp;
    rhs_cell_f<MODE>(c, col[0], col[1], col[2], un, fxm, fz[s], fx, fzp, du[s], dp[s]);
    fz[s] = fzp;
  }
}

// Thread (virtual position index v) -> position (px, py) of a tile of bw = tx/2 stage-B pairs x ty
// rows (round 6), for tiles with positions beyond the threads: whole rows of the R2 tile, each
// row contiguous (wp2 = bw + 2 pairs, so every load and store of a row is one run, as row-major),
// but in the order: stage B's rows 2 .. ty + 1 first, then stage A's ring rows 1 and ty + 2, then
// the load-only rows 0 and ty + 3 -- the last of them beyond the threads (pair_geometry_ok: at most
// PFT_PAIR_NEX, all in row ty + 3).  With 22-pair rows (40 x 20 tile) stage B's 20 rows end at
// thread 439, so the last wave (448 .. 511) holds ring rows only and skips stage B: its SIMD runs 3
// wave-phases a plane where the others run 4, and the extra positions' staging and DMA ride in that
// slack instead of delaying the barrier.  (Stage-B positions compacted to threads 0 .. 399, ring
// columns after them, did the same for pair 2+3 but cost pair 4+5 9%: its rows no longer one run;
// profiles/r06_ab_pair_tile.txt.)  Row-major from row 0 for tiles without extra positions.
__device__ __forceinline__ void pair_pos(int v, int bw, int ty, int& px, int& py)
{
  const int wp2 = bw + 2;
  if (v < ty * wp2) {                                  // stage B's rows
    py = 2 + v / wp2;
    px = v % wp2;
    return;
  }
  v -= ty * wp2;
  if (v < 2 * wp2) {                                   // stage A's ring rows
    py = v < wp2 ? 1 : ty + 2;
    px = v < wp2 ? v : v - wp2;
    return;
  }
  v -= 2 * wp2;                                        // load-only rows
  py = v < wp2 ? 0 : ty + 3;
  px = v < wp2 ? v : v - wp2;
}

template <int N>
using pft_ic = std::integral_constant<int, N>;

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Warray-bounds"
template <int SA, int MODE, bool GLX, int LWP>
__global__ __launch_bounds__(PFT_PBLOCK) __attribute__((amdgpu_waves_per_eu(2))) void merson_pair(PairArgs a,
                                                                                                   pft_consts c)
{
  constexpr bool FLUX = MODE != 10 && MODE != 11;
  constexpr dbl2 zero2 = {0.0, 0.0};
  using LD = PairLds;
#if defined(__HIP_DEVICE_COMPILE__)
  const pft_kptr kbase = (pft_kptr)__builtin_amdgcn_kernarg_segment_ptr();
#endif
  // (the stage-B ring holds rows 1..ty+2 only: PFT_PAIR_HB slots)
  // OPL (pair 4+5 with GLX): stage B's gl input is x's gl, which
  // lA already holds for the same plane -- lB keeps u and p only and stage B reads gl from lA
  // (its z neighbour below from a register: lA's slot of that plane is overwritten by then).  The
  // 22 KiB this frees, with the 22 KiB left over, hold the operands of stage B's outputs (x, K1,
  // K3 of u and p at each stage-B position, 36 KiB): written when they arrive for stage A, read
  // back one plane later by the same thread, instead of their second load from beyond L2 (the
  // re-load: pair 4+5 1.5% slower, 1.80x the algorithmic bytes beyond L2 against 1.11x).
  // (GLB: the same gl sharing in pair 2+3, whose ZREG registers hold stage A's gl inputs at the
  // thread's own position: stage B's gl centre and z neighbours come from there; without it pair
  // 2+3 took 0.341-0.344 against 0.337-0.340 ms)
  constexpr bool GLB = GLX;
  constexpr bool OPL = SA == 4 && GLB;
  constexpr int NBQ = GLB ? 2 : 3;   // lB's fields
  __shared__ __attribute__((aligned(16))) double lA[3][3][2 * PFT_PAIR_H];
  __shared__ __attribute__((aligned(16))) double lB[3][NBQ][2 * PFT_PAIR_HB];
  // (without OPL a 1 x 1 placeholder: its accesses below sit in a branch that is constant-false
  // there, which -Warray-bounds flags per instantiation; an if constexpr would drop the placeholder
  // and shift the LDS layout of every other kernel)
  // lO, then the extra positions' operands of the next plane (x u, p, gl; K1 u, p; K3 u, p), staged
  // by LDS DMA (lX), in one array: the DMA's wave-uniform base lX - 16 (first loader lane) bytes
  // must not fall below the LDS (without OPL a 64-slot pad takes lO's place)
  constexpr int LXOFF = OPL ? 6 * PFT_PAIR_OPN : 64;
  __shared__ __attribute__((aligned(16))) dbl2 lOX[LXOFF + 7 * PFT_PAIR_NEX];
  dbl2(*const lO)[PFT_PAIR_OPN] = reinterpret_cast<dbl2(*)[PFT_PAIR_OPN]>(lOX);
  dbl2* const lX = lOX + LXOFF;
  // the extra positions' acting-pair offsets, set once (the tile's corner x0, y0 is not kept live
  // across the loop for them: pair 4+5 has no register or SGPR to spare)
  __shared__ unsigned lXa[PFT_PAIR_NEX];

  const int TX = a.tx, TY = a.ty, WP2 = TX / 2 + 2, NPOS = WP2 * (TY + 4);
  // inline boundary: the leading workgroups (dispatched first) are the boundary chunks
  const bool bw = (int)blockIdx.x < a.nbw;
  const int lin = bw ? xcd_remap(blockIdx.x, a.nbw) : xcd_remap(blockIdx.x - a.nbw, a.nint);
  const int tile = lin % a.ntile, cq = lin / a.ntile;
  const int chunk = bw ? (a.bends ? (cq ? a.nchunk - 1 : 0) : cq) : a.c0 + cq;
  const bool bshort = bw && !a.bends;   // a two-plane boundary chunk (PFT_K_INLINE)
  const int x0 = (tile % a.ntx) * TX, y0 = (tile / a.ntx) * TY;
  // threads beyond the R2 positions shadow the last one (same loads and LDS writes, no stores)
  const int tt = min((int)threadIdx.x, NPOS - 1);
  int px, py;
  if (LWP == 22 && NPOS > PFT_PBLOCK) {
    pair_pos(tt, TX / 2, TY, px, py);
  } else {
    // no extra positions: row-major over the R2 tile, as measured best there (200^3: the stage-B
    // positions first ran 8% slower, profiles/r06_ab_pair_tile.txt)
    px = tt % WP2;
    py = tt / WP2;
  }
  const int pi = x0 - 2 + 2 * px, pj = y0 - 2 + py;          // position: first cell, row
  // acting pair (in the domain): a mirrored position holds its values (x halves exchanged)
  const int ai = pi < 0 ? 0 : (pi >= a.n1 ? a.n1 - 2 : pi);
  const int aj = pj < 0 ? 0 : (pj >= a.n2 ? a.n2 - 1 : pj);
  // A position outside the domain in x holds the mirror image of its acting pair: the slot stores
  // the acting pair in natural order (16-byte stores and loads, no per-lane swap), and the
  // neighbour reading it takes the other cell (mirrored pair (-2, -1) = (v1, v0) holds (v0, v1):
  // cell -1 is its even cell; (n1, n1 + 1) holds (v[n1-2], v[n1-1]): cell n1 is its odd cell).
  auto mir = [&](int col) -> bool { const int c0 = x0 - 2 + 2 * col; return c0 < 0 || c0 >= a.n1; };
  const int pxa = (ai - x0 + 2) / 2;                          // the acting pair's column
  const int xmcA = mir(pxa - 1) ? 0 : 1, xpcA = mir(pxa + 1) ? 1 : 0;
  const int xmcB = mir(px - 1) ? 0 : 1, xpcB = mir(px + 1) ? 1 : 0;
  const unsigned apo = (unsigned)(aj * a.n1 + ai);
  // byte offset of the acting pair in plane m of a field, from the PairArgs pointers
  auto pbo = [&](int m) -> unsigned { return ((unsigned)(m + 2) * (unsigned)a.plane + apo) * 8u; };
  const int posA = PFT_PAIR_PADP + py * LWP + px;              // this position's slot in lA
  const int posB = PFT_PAIR_PADP + (py - 1) * LWP + px;        // ... in lB (rows 1..ty+2)
  const int actA = PFT_PAIR_PADP + (aj - y0 + 2) * LWP + (ai - x0 + 2) / 2;   // the acting pair in lA
  const bool isA = py >= 1 && py <= TY + 2;
  const bool isB = (int)threadIdx.x < NPOS && px >= 1 && px <= TX / 2 && py >= 2 && py <= TY + 1 &&
                   pi < a.n1 && pj < a.n2;
  const int ob = (py - 2) * (TX / 2) + px - 1;                // this stage-B position's slot in lO
  // positions beyond the threads (NPOS > PFT_PBLOCK: pair_geometry_ok puts them all in the last
  // ring row ty + 3, the tail of pair_pos's order): the last NPOS - PFT_PBLOCK threads (lanes
  // 64 - NEX .. 63 of the last wave, themselves load-only positions) load one each too, by LDS DMA
  // into lX one plane ahead like their own look-ahead, and store its stage-A input into lA with
  // their own.  Everything about it is recomputed where used from the thread index and the phase's
  // kernel arguments (mostly scalar): the kernel holds no register for it across the loop (pair
  // 4+5 is at 256 VGPRs).
  auto nex = [&](const PairArgs& A) { return (A.tx / 2 + 2) * (A.ty + 4) - PFT_PBLOCK; };
  // the loaders are lanes 64 - NEX .. 63 of the last wave; inside the z-loop they are found from
  // the wave's index (one SGPR) and the lane index (mbcnt, recomputed): keeping threadIdx.x live
  // across the loop for them cost pair 4+5 a spilled VGPR
  const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  auto lane = [&]() {
    int l;  // volatile: recomputed where used, so nothing derived from it is hoisted out of the loop
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
  };
  // (only tiles wider than 20 cells have them: the 12-pair pitch compiles the extras out)
  auto is_x = [&](const PairArgs& A) { return LWP == 22 && wid == PFT_PBLOCK / 64 - 1 && lane() >= 64 - nex(A); };
  // the extra position's column (row ty + 3) and its acting pair's offset in a plane
  auto px_x = [&](const PairArgs& A) { return lane() - 64 + (A.tx / 2 + 2); };
  auto apo_x = [&](const PairArgs& A) { return lXa[lane() - (64 - nex(A))]; };
  auto pos_x = [&](const PairArgs& A) { return PFT_PAIR_PADP + (A.ty + 3) * LWP + px_x(A); };
  auto pboe = [&](const PairArgs& A, int m) -> unsigned { return ((unsigned)(m + 2) * (unsigned)A.plane + apo_x(A)) * 8u; };
  // the DMA of plane m's operands of the extra position into lX (this lane: slot xs of each array)
  auto dma = [&](const PairArgs& A, int m) {
    const unsigned bo = pboe(A, m);
    const unsigned l0 = (unsigned)(size_t)((__attribute__((address_space(3))) dbl2*)lX) -
                        16u * (unsigned)(64 - nex(A));       // lane 64 - NEX -> slot 0
    const unsigned fb = (unsigned)A.fs * 8u;                  // a field's bytes (pft_slab_pair_ok: 3 fb < 4 GiB)
#pragma unroll
    for (int q = 0; q < 3; ++q) lds_dma16(l0 + (0 + q) * 16 * PFT_PAIR_NEX, A.x, bo + q * fb);
#pragma unroll
    for (int q = 0; q < 2; ++q) lds_dma16(l0 + (3 + q) * 16 * PFT_PAIR_NEX, A.k1, bo + q * fb);
    if (SA == 4) {
#pragma unroll
      for (int q = 0; q < 2; ++q) lds_dma16(l0 + (5 + q) * 16 * PFT_PAIR_NEX, A.k3, bo + q * fb);
    }
  };
  // stage A's input of the extra position from the staging (after pair_x_wait), field by field,
  // into the ring slot `slot`
  auto xstore = [&](const PairArgs& A, int slot) {
    const int xs = lane() - (64 - nex(A));                   // this loader's slot in lX (0 .. NEX - 1)
    const int pe = pos_x(A);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      PairRaw t;
      t.x[q] = lX[(0 + q) * PFT_PAIR_NEX + xs];
      if (q < 2) {
        t.k1[q] = lX[(3 + q) * PFT_PAIR_NEX + xs];
        if (SA == 4) t.k3[q] = lX[(5 + q) * PFT_PAIR_NEX + xs];
      }
      LD::st(lA[slot][q], pe, pair_in_A<SA, GLX>(A, q, t));
    }
  };

  const int kb = bshort ? chunk * (a.n3 - 2) : a.k_begin + chunk * a.kz;
  const int ke = bshort ? kb + 2 : min(kb + a.kspan, a.k_end);
  const int n3 = a.n3;
  const bool wlo = !a.has_below, whi = !a.has_above;         // walls (equation.c:164-183)
  // stage-A planes [mA0, mA1]: the chunk's planes and one on each side -- at a slab interface
  // the ghost plane (the neighbour's boundary plane, recomputed), at a wall none
  const int mA0 = kb > 0 ? kb - 1 : (wlo ? 0 : -1);
  const int mA1 = ke < n3 ? ke : (whi ? n3 - 1 : n3);
  const int mlast = min(mA1 + 1, whi ? n3 - 1 : n3 + 1);     // last stage-A input plane
  const int mfirst = wlo ? 0 : -2;                           // first stage-A input plane

  double m = 0.0;
  bool nf = false;
  // Operands in registers: those of plane mm (stage B's input), mm + 1 (landed: stage A's input)
  // and mm + 2 (in flight), rotating through R[0..2]; stage B's outputs (4+5) need plane mm - 1's
  // again: from lO (OPL), else re-loaded after stage A (in registers they would spill).
  // Plane p's LDS ring slot is (p - mA0) mod 3 and the loop is unrolled three times, so every ring
  // slot -- and with the fixed row pitch every LDS offset -- is a compile-time constant, and the
  // register rotation needs no copies.
  PairRaw R[3];
  dbl2 KA[3][2];        // stage A's K (u, p) of the last three planes, rotating with R
  // ZREG (pair 2+3, which has the registers: 218 VGPRs with it): stage A's inputs at this
  // thread's own position, plane by ring slot, kept in registers beside their LDS copies -- stage
  // A reads its z neighbours and centre from here instead of from LDS (measured: pair 2+3 0.362 ->
  // 0.354 ms, 200^3 +1.0%; profiles/r04b_ab_small_grids_and_layouts.txt ab4q).  Pair 4+5 has no
  // registers for it (256 VGPRs in use).
  constexpr bool ZREG = SA == 2;
  dbl2 IA[3][3];
  dbl2 glm = zero2;     // GLB: gl's input at this position, plane mm - 2 (stage B's z neighbour below)
  FaceT fzA[2], fzB[2];

  // prologue: stage A's input of planes mA0 - 1 (if any) and mA0 into the ring (slots 2 and 0);
  // operands of mA0 kept, of mA0 + 1 in flight.  (kb >= ke: an empty chunk, which still takes
  // part in the error norm's workgroup count below)
  if (is_x(a)) {
    const int ajx = min(y0 - 2 + a.ty + 3, a.n2 - 1);
    const int aix = min(max(x0 - 2 + 2 * px_x(a), 0), a.n1 - 2);
    lXa[(int)threadIdx.x - (PFT_PBLOCK - nex(a))] = (unsigned)(ajx * a.n1 + aix);
  }
  if (kb < ke) {
    dbl2 ia0[3], iam[3];
    pair_load<SA>(a, pbo(mA0), R[0]);
    if (mA0 > mfirst) {
      PairRaw t;
      pair_load<SA>(a, pbo(mA0 - 1), t);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        iam[q] = pair_in_A<SA, GLX>(a, q, t);
        LD::st(lA[2][q], posA, iam[q]);
        if (ZREG) IA[2][q] = iam[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      ia0[q] = pair_in_A<SA, GLX>(a, q, R[0]);
      LD::st(lA[0][q], posA, ia0[q]);
      if (ZREG) IA[0][q] = ia0[q];
      if (mA0 == mfirst) {
        // bottom wall: plane -1 mirrors plane 0 (equation.c:164-174), also in the ring slot of
        // plane -1, so that the z-loop reads its z neighbours without selects
        iam[q] = ia0[q];
        LD::st(lA[2][q], posA, ia0[q]);
        if (ZREG) IA[2][q] = ia0[q];
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) fzA[s] = face_of(c, iam[1][s], iam[2][s], iam[0][s], ia0[1][s], ia0[2][s], ia0[0][s], FLUX);
    if (is_x(a)) {
      // the extra position: planes mA0 - 1 and mA0 as the others' (loaded here), mA0 + 1 by DMA
      PairRaw t;
      if (mA0 > mfirst) {
        pair_load<SA>(a, pboe(a, mA0 - 1), t);
#pragma unroll
        for (int q = 0; q < 3; ++q) LD::st(lA[2][q], pos_x(a), pair_in_A<SA, GLX>(a, q, t));
      }
      pair_load<SA>(a, pboe(a, mA0), t);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const dbl2 v = pair_in_A<SA, GLX>(a, q, t);
        LD::st(lA[0][q], pos_x(a), v);
        if (mA0 == mfirst) LD::st(lA[2][q], pos_x(a), v);
      }
      if (mA0 + 1 <= mlast) dma(a, mA0 + 1);                // consumed in the first step's stage-B slot
    }
    if (mA0 + 1 <= mlast) pair_load<SA>(a, pbo(mA0 + 1), R[1]);
    KA[2][0] = KA[2][1] = zero2;
    __syncthreads();
  }

  // one z-step: stage A at plane mm, stage B at plane mm - 1; false after the chunk's last one
  auto step = [&](auto ph, int mm, PairRaw& rc, PairRaw& rn, PairRaw& rnn) -> bool {
    constexpr int PH = decltype(ph)::value;
    constexpr int sA = PH, sAm = (PH + 2) % 3, sAp = (PH + 1) % 3;   // ring slots of planes mm, mm-1, mm+1
    {
      PFT_PAIR_BIND(A0, C0);
      (void)C0;
      if (GLB) glm = ZREG ? IA[sAp][2] : LD::ld(lA[sAp][2], posA);   // plane mm - 2, before mm + 1 replaces it
      // stage A's input of plane mm + 1 (own pair: read back by this thread in this iteration;
      // x/y neighbours: in the next one, behind the barrier), and the look-ahead load of plane
      // mm + 2.  Both unconditional -- beyond mlast the load re-reads plane mlast and the store
      // lands in the ring slot of plane mm - 2, which nobody reads any more -- so that no branch
      // separates a load from its use: with the loads under a branch the compiler's s_waitcnt
      // placement lost track of them and stage A waited for the look-ahead it had just issued.
      if (mm + 1 <= mlast) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const dbl2 v = pair_in_A<SA, GLX>(A0, q, rn);
          LD::st(lA[sAp][q], posA, v);
          if (ZREG) IA[sAp][q] = v;
        }
      }
      if (mm + 2 <= mlast) pair_load<SA>(A0, pbo(mm + 2), rnn);          // look-ahead
    }
    const int kB = mm - 1;                                   // stage B's plane
    PairRaw ro;
    {
      PFT_PAIR_BIND(A1, C1);
      // The two waves of a SIMD (w and w + 4) run the same phase between two barriers, so their
      // stalls coincide.  Waves 0-3 get issue precedence in stage A (pair 2+3: waves 4-7 in stage
      // B, pair 4+5: nobody), so the two drift apart and fill each other's stalls.  Measured (A/B,
      // one box): pair 4+5 0.496 -> 0.480 ms; pair 2+3 0.425 -> 0.403 ms.
      if ((threadIdx.x >> 8) == 0) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(0);
      dbl2 (&ka)[2] = KA[PH];
      ka[0] = ka[1] = zero2;
      if (mm <= mA1 && isA) {
        // stage A at plane mm, evaluated as the acting pair's thread does
        if (mm == n3 - 1 && whi) {
          // top wall: the ring slot of plane n3 holds the ghost values -- Dirichlet u (equation.c:
          // 175-183), p and gl mirrored -- at this position (its own z neighbour only)
#pragma unroll
          for (int q = 1; q < 3; ++q) LD::st(lA[sAp][q], posA, LD::ld(lA[sA][q], posA));
          LD::st(lA[sAp][0], posA, dbl2{A1.T_topA, A1.T_topA});
          if (ZREG) {
            IA[sAp][1] = IA[sA][1];
            IA[sAp][2] = IA[sA][2];
            IA[sAp][0] = dbl2{A1.T_topA, A1.T_topA};
          }
        }
        dbl2 zc[3], zm[3], zp[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          zc[q] = ZREG ? IA[sA][q] : LD::ld(lA[sA][q], posA);
          zm[q] = ZREG ? IA[sAm][q] : LD::ld(lA[sAm][q], posA);
          zp[q] = ZREG ? IA[sAp][q] : LD::ld(lA[sAp][q], posA);
        }
        double du[2], dp[2];
        const double* nz = A1.noise ? A1.noise + (long)mm * A1.plane + (long)apo : nullptr;
        pair_rhs<MODE, LWP>(C1, lA[sA][0], lA[sA][1], lA[sA][2], actA, xmcA, xpcA, zm, zc, zp, nz, fzA, du, dp);
        ka[0] = dbl2{du[0], du[1]};
        ka[1] = dbl2{dp[0], dp[1]};
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
          const dbl2 ib = pair_in_B<SA, GLX>(A1, q, rc, q < 2 ? ka[q < 2 ? q : 0] : zero2);
          LD::st(lB[sA][q], posB, ib);
          if (mm == 0 && wlo) LD::st(lB[sAm][q], posB, ib);   // bottom wall: plane -1 mirrors plane 0
        }
      }
    }
    {
      PFT_PAIR_BIND(A2, C2);
      if (SA == 4) __builtin_amdgcn_s_setprio(0);
      else if ((threadIdx.x >> 8) == 0) __builtin_amdgcn_s_setprio(0);
      else __builtin_amdgcn_s_setprio(2);
      // operands of plane kB for stage B's outputs (4+5).  OPL: from lO.  Otherwise loaded a
      // second time, after stage A (in registers they would need ~60 VGPRs more than the 255 in
      // use), and NOT an L2 hit: their first load was the look-ahead three planes earlier, and
      // three planes of the ring's operands of the ~32 workgroups of an XCD (~5 MB) exceed its
      // 4 MB L2 -- the Infinity Cache serves them (PMC: 1.80x the algorithmic bytes beyond L2
      // with the re-load, 1.11x with lO; pair 4+5 -1.5%: DESIGN.md section 5)
      // (GLX: gl's x(t+h) is not stored, XN holds it: gl's x is not needed)
      // (unconditional, as the look-ahead: every lane's acting pair is in the domain)
      if (OPL) {
        // plane kB's operands from lO, then plane mm's into the same slot (this thread's own; LDS
        // accesses of a wave stay in order)
        if (kB >= kb && isB) {
          ro.x[0] = lO[0][ob];
          ro.x[1] = lO[1][ob];
          ro.k1[0] = lO[2][ob];
          ro.k1[1] = lO[3][ob];
          ro.k3[0] = lO[4][ob];
          ro.k3[1] = lO[5][ob];
        }
        if (isB && mm >= kb && mm < ke) {
          lO[0][ob] = rc.x[0];
          lO[1][ob] = rc.x[1];
          lO[2][ob] = rc.k1[0];
          lO[3][ob] = rc.k1[1];
          lO[4][ob] = rc.k3[0];
          lO[5][ob] = rc.k3[1];
        }
      } else if (SA == 4 && kB >= kb && isB) {
        pair_load<SA, !GLX>(A2, pbo(kB), ro);
      }
      if (kB >= kb && isB) {
        constexpr int sB = (PH + 2) % 3, sBm = (PH + 1) % 3, sBp = PH;   // slots of planes kB, kB-1, kB+1
        const int lo = posB;
        if (kB == n3 - 1 && whi) {
          // top wall: the ghost values of plane n3 at this position (as in stage A above)
#pragma unroll
          // (GLB: gl's ghost is in lA's slot of plane n3, from stage A's top wall)
          for (int q = 1; q < NBQ; ++q) LD::st(lB[sBp][q], lo, LD::ld(lB[sB][q], lo));
          LD::st(lB[sBp][0], lo, dbl2{A2.T_topB, A2.T_topB});
        }
        dbl2 zc[3], zm[3], zp[3];
#pragma unroll
        for (int q = 0; q < NBQ; ++q) {
          zc[q] = LD::ld(lB[sB][q], lo);
          zm[q] = LD::ld(lB[sBm][q], lo);
          zp[q] = LD::ld(lB[sBp][q], lo);
        }
        if (GLB) {
          zc[2] = ZREG ? IA[sB][2] : LD::ld(lA[sB][2], posA);
          zm[2] = glm;
          zp[2] = ZREG ? IA[sBp][2] : LD::ld(lA[sBp][2], posA);
        }
        if (kB == kb) {
          // the z-face below the chunk's first stage-B plane
#pragma unroll
          for (int s = 0; s < 2; ++s)
            fzB[s] = face_of(C2, zm[1][s], zm[2][s], zm[0][s], zc[1][s], zc[2][s], zc[0][s], FLUX);
        }
        double du[2], dp[2];
        const unsigned e0 = pbo(kB);
        const double* nz = A2.noise ? A2.noise + (long)kB * A2.plane + (long)apo : nullptr;
        // (GLB: gl's plane from lA, whose rows start one row earlier: slot lo + LWP there)
        const double* lBgl = GLB ? &lA[sB][2][2 * LWP] : &lB[sB][NBQ - 1][0];
        pair_rhs<MODE, LWP>(C2, lB[sB][0], lB[sB][1], lBgl, lo, xmcB, xpcB, zm, zc, zp, nz, fzB, du, dp);
        if (SA == 2) {
          stb(A2.out, e0, dbl2{du[0], du[1]});                   // K3 (hybrid2.c:412-429)
          stb(A2.out + A2.fs, e0, dbl2{dp[0], dp[1]});
        } else {
          const dbl2(&kao)[2] = KA[(PH + 2) % 3];              // stage A's K (K4) at plane kB
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const dbl2 K = q == 0 ? dbl2{du[0], du[1]} : dbl2{dp[0], dp[1]};
            const dbl2 k1 = ro.k1[q], k3 = ro.k3[q], k4 = kao[q];
            const double em = q == 0 ? A2.em0 : A2.em1;
            dbl2 r;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const double ev = em * fabs(0.2 * k1[s] - 0.9 * k3[s] + 0.8 * k4[s] - 0.1 * K[s]);   // :521
              if (ev > m) m = ev;                                                            // NaN never wins
              nf |= !isfinite(ev);
              r[s] = ro.x[q][s] + A2.coef * (0.5 * (k1[s] + K[s]) + 2.0 * k4[s]);            // :667
            }
            stb(A2.out + q * A2.fs, e0, r);
          }
          // gl: x(t+h) = x + coef (0.5 (0.0 + 0.0) + 2.0 0.0), stored unless XN already holds it
          if (!GLX && !A2.gl_keep) stb(A2.out + 2 * A2.fs, e0, dbl2{ro.x[2][0] + A2.glX, ro.x[2][1] + A2.glX});
        }
      }
    }
    {
      PFT_PAIR_BIND(A3, C3);
      (void)C3;
      if (is_x(A3)) {
        // the extra positions, in the last wave's stage-B slot (it holds no stage-B position, its
        // SIMD has a wave-phase to spare: pair_pos), after stage B, where few registers are live:
        // plane mm + 1's operands from the staging (its DMA went out an iteration ago; the wait for
        // everything this wave issued is only the last wave's), stage A's input into lA, then plane
        // mm + 2's DMA -- not in the chunk's last step, so that no DMA is left outstanding when the
        // workgroup ends
        if (mm + 1 <= mlast) {
          pair_x_wait<0>();
          xstore(A3, (PH + 1) % 3);
        }
        if (mm + 2 <= mlast && mm < ke) dma(A3, mm + 2);
      }
    }
    if (mm == ke) return false;
    __syncthreads();
    return true;
  };

  if (kb < ke) {
    for (int mm = mA0;; mm += 3) {
      if (!step(pft_ic<0>{}, mm, R[0], R[1], R[2])) break;
      if (!step(pft_ic<1>{}, mm + 1, R[1], R[2], R[0])) break;
      if (!step(pft_ic<2>{}, mm + 2, R[2], R[0], R[1])) break;
    }
  }

  if (SA == 4) {
    __shared__ double red[PFT_PBLOCK / 64];
    __shared__ int rnf[PFT_PBLOCK / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(m, off, 64);
      if (ov > m) m = ov;
    }
    const int anynf = __any(nf);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[w] = m;
      rnf[w] = anynf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double bm = red[0];
      int bnf = rnf[0];
      for (int q = 1; q < PFT_PBLOCK / 64; ++q) {
        if (red[q] > bm) bm = red[q];
        bnf |= rnf[q];
      }
      // gl's error-norm term: the same constant at every cell (its K's are literal zeros)
      if (a.evgl > bm) bm = a.evgl;
      bnf |= !isfinite(a.evgl);
      if (a.part) eps_store_part(a.part, bm, bnf);
      else eps_arrive(bm, bnf, a.shards, a.eps_bits, a.nonfinite, a.pub, a.pub_count);
    }
  }
  if (bw) {
    // an inline boundary workgroup: every wave's stores done, then one lane writes the XCD's L2
    // back (system scope: the copy engines read memory, not this L2) and counts the workgroup; the
    // copies wait for the count (bnd_trigger_kernel) while the interior workgroups go on
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_fetch_add(a.bdone, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
#pragma clang diagnostic pop

// the copy-engine exchange of an inline boundary (PFT_K_INLINE): this one-wave kernel ends once the
// boundary workgroups of the launch have counted themselves (*bdone >= target, monotonic), so the
// plane copies queued behind it on the comm stream start while that launch's interior still runs.
// It sits on a CU the boundary workgroups freed; nothing it waits for depends on another rank.
__global__ __launch_bounds__(64) void bnd_trigger_kernel(const unsigned long long* bdone, unsigned long long target)
{
  if (threadIdx.x == 0)
    while (__hip_atomic_load(bdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(2);
}

// ------------------------------------------------------------------------------------------
// f1: the default Params' initial condition and the glass beads on the device (pft_slab_ic_default)

struct IcDev {
  double* x;             // X
  double* xn;            // XN (the same values)
  long fs;
  int n1, n2, n3, plane;
  const double* tab;     // tx1 tx2 px2 xb [n1], ty1 ty2 py2 yb [n2], tz1 tz2 pz zb [n3], beads 3*nb
  const int* poff;       // [n3 + 1]
  const int* pbead;
  int nbeads;
  double u0, r2, s, R, reach2;
  unsigned int* unclean;
  int overlay;           // 1: the beads over X's gl (an IC already in X, e.g. ic_prog_kernel's); u, p kept
};

// one thread per interior node: pft_model_ic_default (Params:9-21 as the reference's evaluator
// computes them: u = 293.15; p = 1 inside the ice disc, else 0; gl the max of the six wall terms in
// the formula's order) and overlay_beads (equation.c:507-530: gl = max(gl, 0.5 (1 - tanh(s (|x -
// b| + 1e-10 - R))))), every operation the host's in the host's order, no contraction
__global__ __launch_bounds__(256) void ic_default_kernel(IcDev a)
{
  const long n = (long)a.plane * a.n3;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int k = (int)(e / a.plane);
  const int r = (int)(e - (long)k * a.plane);
  const int j = r / a.n1, i = r - j * a.n1;
  const double* X = a.tab;
  const double* Y = X + 4 * a.n1;
  const double* Z = Y + 4 * a.n2;
  const double* B = Z + 4 * a.n3;
  const long o = (long)(k + 1) * a.plane + r;
  double p = 0.0, gl;
  if (a.overlay) {
    gl = a.x[2 * a.fs + o];
  } else {
    p = (Z[2 * a.n3 + k] != 0.0 && X[2 * a.n1 + i] + Y[2 * a.n2 + j] < a.r2) ? 1.0 : 0.0;
    gl = Z[k];
    gl = gl > Z[a.n3 + k] ? gl : Z[a.n3 + k];           // evmax (ee_wrapper.cc:246-250), in order
    gl = gl > X[i] ? gl : X[i];
    gl = gl > Y[j] ? gl : Y[j];
    gl = gl > X[a.n1 + i] ? gl : X[a.n1 + i];
    gl = gl > Y[a.n2 + j] ? gl : Y[a.n2 + j];
  }
  if (a.nbeads) {
    const double x = X[3 * a.n1 + i], y = Y[3 * a.n2 + j], z = Z[3 * a.n3 + k];
    for (int t = a.poff[k]; t < a.poff[k + 1]; ++t) {
      const int b = a.pbead[t];
      const double v1 = x - B[3 * b], v2 = y - B[3 * b + 1], v3 = z - B[3 * b + 2];
      const double d2 = v1 * v1 + v2 * v2 + v3 * v3;
      if (d2 > a.reach2) continue;
      const double nrm = sqrt(d2) + 1E-10;
      const double phf = 0.5 * (1.0 - pft_tanh(a.s * (nrm - a.R)));
      if (gl < phf) gl = phf;
    }
  }
  if (!a.overlay) {
    a.x[o] = a.u0;
    a.x[a.fs + o] = p;
    a.xn[o] = a.u0;
    a.xn[a.fs + o] = p;
  }
  a.x[2 * a.fs + o] = gl;
  a.xn[2 * a.fs + o] = gl;
  if (gl != gl || (gl == 0.0 && signbit(gl))) atomicOr(a.unclean, 1u);
}

// f1 for any icond formula (pft_ic_compile): one thread per interior node runs the compiled
// residual program (csrc/pft_ic_ops.h, the host's operators) on the node's u, p, gl in X and the
// host-evaluated per-axis tables, into field q of X and XN -- as pft_ic_eval does on the host array
struct IcProgDev {
  double* x;
  double* xn;
  long fs;
  int n1, n2, n3, plane, q, n;
  const int* op;
  const double* arg;
  const int* taxis;
  const long* toff;
  const double* tval;
  const unsigned char* terr;
};

__global__ __launch_bounds__(256) void ic_prog_kernel(IcProgDev a)
{
  const long n = (long)a.plane * a.n3;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int k = (int)(e / a.plane);
  const int r = (int)(e - (long)k * a.plane);
  const int j = r / a.n1, i = r - j * a.n1;
  const long o = (long)(k + 1) * a.plane + r;
  const double node[3] = {a.x[o], a.x[a.fs + o], a.x[2 * a.fs + o]};
  const double v = pft_ic_run(a.n, a.op, a.arg, node, a.taxis, a.toff, a.tval, a.terr, i, j, k);
  a.x[a.q * a.fs + o] = v;
  a.xn[a.q * a.fs + o] = v;
}

// ------------------------------------------------------------------------------------------
// layout conversion kernels (host padded layout, ghost thickness 2 <-> device layout)

__global__ void publish_kernel(unsigned long long* __restrict__ d, unsigned long long* host)
{
  host[0] = d[0];
  host[1] = d[1];
  d[0] = 0;              // ready for the next step's error norm (no separate fill)
  d[1] = 0;
  __threadfence_system();
}

__global__ void pack_kernel(const double* __restrict__ host, double* __restrict__ dev, int n1, int n2,
                            int n3, long fs, long S)
{
  // planes -1..n3 of every field (ghost planes included)
  const long plane = (long)n1 * n2;
  const long total = 3L * (n3 + 2) * plane;
  const int N1 = n1 + 4, N2 = n2 + 4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int q = (int)(e / ((n3 + 2) * plane));
    const long r = e - (long)q * (n3 + 2) * plane;
    const int kk = (int)(r / plane);          // 0..n3+1 = k+1
    const long c = r - (long)kk * plane;
    const int j = (int)(c / n1), i = (int)(c - (long)j * n1);
    dev[q * fs + r] = host[q * S + (long)(kk + 1) * N1 * N2 + (long)(j + 2) * N1 + (i + 2)];
  }
}

__global__ void unpack_kernel(const double* __restrict__ dev, double* __restrict__ host, int n1, int n2,
                              int n3, long fs, long S)
{
  // interior planes only
  const long plane = (long)n1 * n2;
  const long total = 3L * n3 * plane;
  const int N1 = n1 + 4, N2 = n2 + 4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int q = (int)(e / (n3 * plane));
    const long r = e - (long)q * n3 * plane;
    const int k = (int)(r / plane);
    const long c = r - (long)k * plane;
    const int j = (int)(c / n1), i = (int)(c - (long)j * n1);
    host[q * S + (long)(k + 2) * N1 * N2 + (long)(j + 2) * N1 + (i + 2)] = dev[q * fs + (long)(k + 1) * plane + c];
  }
}

// ------------------------------------------------------------------------------------------
// generic chunk-table combines (host-staged path for unregistered right-hand sides)

__global__ void flat_combine_kernel(int stage, int n_chunks, const int* __restrict__ cstart,
                                    const int* __restrict__ csize, const double* __restrict__ cmult,
                                    double coef, double h, const double* x, const double* k1,
                                    const double* k2, const double* k3, const double* k4,
                                    const double* k5, double* out, unsigned long long* eps_bits,
                                    unsigned int* nonfinite)
{
  double m = 0.0;
  bool nf = false;
  for (int ch = blockIdx.x; ch < n_chunks; ch += gridDim.x) {
    const long s0 = cstart[ch];
    const int n = csize[ch];
    const double mult = cmult ? cmult[ch] : 1.0;
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
      const long e = s0 + t;
      switch (stage) {
        case 1: out[e] = k1[e] * coef + x[e]; break;                              // :388
        case 2: out[e] = (k1[e] + k2[e]) * coef + x[e]; break;                    // :408
        case 3: out[e] = (k1[e] + 3.0 * k3[e]) * coef + x[e]; break;              // :428
        case 4: out[e] = (0.5 * k1[e] - 1.5 * k3[e] + 2.0 * k4[e]) * h + x[e]; break;  // :449
        case 5: {
          const double ev = mult * fabs(0.2 * k1[e] - 0.9 * k3[e] + 0.8 * k4[e] - 0.1 * k5[e]);
          if (ev > m) m = ev;
          nf |= !isfinite(ev);
        } break;
        case 6: out[e] += coef * (0.5 * (k1[e] + k5[e]) + 2.0 * k4[e]); break;    // :667
      }
    }
  }
  if (stage == 5) {
    __shared__ double red[PFT_BLOCK / 64];
    __shared__ int rnf[PFT_BLOCK / 64];
    for (int off = 32; off > 0; off >>= 1) {
      const double o = __shfl_xor(m, off, 64);
      if (o > m) m = o;
    }
    const int anynf = __any(nf);
    if ((threadIdx.x & 63) == 0) {
      red[threadIdx.x >> 6] = m;
      rnf[threadIdx.x >> 6] = anynf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double bm = red[0];
      int bnf = rnf[0];
      for (int k = 1; k < (int)(blockDim.x / 64); ++k) {
        if (red[k] > bm) bm = red[k];
        bnf |= rnf[k];
      }
      if (bm > 0.0) atomicMax(eps_bits, (unsigned long long)__double_as_longlong(bm));
      if (bnf) atomicOr(nonfinite, 1u);
    }
  }
}

// ------------------------------------------------------------------------------------------
// ipc transport (pft_comm.h): this slab's boundary planes go straight into the z-neighbours' ghost
// planes (IPC-mapped device memory, on this GPU or over xGMI), then the last workgroup publishes the
// exchange's sequence number in the neighbours' flag words; each side's stream waits for its own
// flags (hipStreamWaitValue64), so the next stage starts only once both ghost planes are in.

struct PutArgs {
  const double* src;          // this slab's buffer (one role)
  long fs;
  int plane, n3, f0, nf;
  double* dlo;                // the neighbour below: its top ghost plane (n3' + 1) of field 0, or null
  long dlo_fs;
  double* dhi;                // the neighbour above: its bottom ghost plane (0) of field 0, or null
  long dhi_fs;
  int deep;                   // 1: also the second planes, into the neighbours' far ghost planes
  double* flo;                // the neighbour below's far plane above (n3' + 2) of field 0
  double* fhi;                // the neighbour above's far plane below (-1) of field 0
};

__global__ __launch_bounds__(256) void halo_put_kernel(PutArgs a)
{
  const long n = (long)a.nf * a.plane;   // doubles per side and depth
  const long tot = (a.deep ? 4 : 2) * n;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
    const int part = (int)(e / n);       // 0: plane 1 down, 1: plane n3 up, 2: plane 2 down (far), 3: plane n3-1 up (far)
    const long r = e - part * n;
    const int f = (int)(r / a.plane);
    const long c = r - (long)f * a.plane;
    const int q = a.f0 + f;
    if (part == 0) {
      if (a.dlo) a.dlo[q * a.dlo_fs + c] = a.src[q * a.fs + (long)a.plane + c];
    } else if (part == 1) {
      if (a.dhi) a.dhi[q * a.dhi_fs + c] = a.src[q * a.fs + (long)a.n3 * a.plane + c];
    } else if (part == 2) {
      if (a.flo) a.flo[q * a.dlo_fs + c] = a.src[q * a.fs + 2L * a.plane + c];
    } else {
      if (a.fhi) a.fhi[q * a.dhi_fs + c] = a.src[q * a.fs + (long)(a.n3 - 1) * a.plane + c];
    }
  }
}

// Staged receive (pft_slab_halo_wait): the planes the neighbours put into this slab's receive
// buffer rbuf (uncached; two slots by the exchange's parity, each [side][depth][field][plane], side
// 0 from below, 1 from above; depth 0 the ghost plane, 1 the far ghost plane) copied into the ghost planes of buffer dst, fields
// [f0, f0 + nf), for the sides in `sides` (bit 0 below, bit 1 above)
struct RecvArgs {
  const double* rbuf;
  double* dst;                // the buffer (pft_slab_buffer layout: plane 0 = ghost below)
  long fs;
  int plane, n3, f0, nf, depth, sides;
};

__global__ __launch_bounds__(256) void halo_recv_kernel(RecvArgs a)
{
  const long n = (long)a.nf * a.plane;
  const long tot = 4L * n;              // (side, depth) parts, skipped where not received
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
    const int part = (int)(e / n);
    const int side = part >> 1, depth = part & 1;
    if (!((a.sides >> side) & 1) || depth >= a.depth) continue;
    const long r = e - part * n;
    const int f = (int)(r / a.plane);
    const long c = r - (long)f * a.plane;
    const int q = a.f0 + f;
    const long pl = side == 0 ? (depth == 0 ? 0L : -1L) : (long)a.n3 + 1 + depth;
    a.dst[q * a.fs + pl * a.plane + c] = a.rbuf[((long)(side * 2 + depth) * 3 + q) * a.plane + c];
  }
}

// The receiving side of an exchange in ONE launch (pft_slab_halo_wait): thread 0 of every workgroup
// waits until both flag words reach seq (system-scope atomic loads of uncached memory: never served
// from a cache), then -- staged receive -- the workgroups copy the receive buffer into the ghost
// planes (halo_recv_kernel's loop).  It replaces hipStreamWaitValue64 per flag (the runtime runs each
// as a kernel of its own, ~3 us apiece) and the separate receive launch.  Every wave exits: the
// flags come from the neighbours, or from the slab itself when a wait times out (slab_timed_out
// releases them past every sequence number).
struct WaitArgs {
  const unsigned long long* f0;   // flag from below, or null
  const unsigned long long* f1;   // flag from above, or null
  unsigned long long seq;
  int recv;                       // 1: then copy r
  RecvArgs r;
};

__global__ __launch_bounds__(256) void halo_wait_kernel(WaitArgs a)
{
  if (threadIdx.x == 0) {
    if (a.f0)
      while (__hip_atomic_load(a.f0, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) __builtin_amdgcn_s_sleep(2);
    if (a.f1)
      while (__hip_atomic_load(a.f1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) __builtin_amdgcn_s_sleep(2);
  }
  __syncthreads();
  if (!a.recv) return;
  const RecvArgs& r = a.r;
  const long n = (long)r.nf * r.plane;
  const long tot = 4L * n;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < tot; e += (long)gridDim.x * blockDim.x) {
    const int part = (int)(e / n);
    const int side = part >> 1, depth = part & 1;
    if (!((r.sides >> side) & 1) || depth >= r.depth) continue;
    const long rr = e - part * n;
    const int f = (int)(rr / r.plane);
    const long c = rr - (long)f * r.plane;
    const int q = r.f0 + f;
    const long pl = side == 0 ? (depth == 0 ? 0L : -1L) : (long)r.n3 + 1 + depth;
    r.dst[q * r.fs + pl * r.plane + c] = r.rbuf[((long)(side * 2 + depth) * 3 + q) * r.plane + c];
  }
}

// raises the neighbours' flags once the kernels before it on the stream (the put, or a stage
// kernel that stored its boundary planes into the neighbours' ghost planes) have completed: their
// stores are released at kernel end; with a neighbour on another GPU a system-scope fence first
// (the flag must not overtake the plane over xGMI).  One thread, vector atomics only.
__global__ void halo_signal_kernel(unsigned long long* slo, unsigned long long* shi, unsigned long long seq,
                                   int remote)
{
  if (threadIdx.x != 0) return;
  if (remote) __threadfence_system();
  if (slo) __hip_atomic_store(slo, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (shi) __hip_atomic_store(shi, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------------------------------
// calibration probe: a plain 8-byte-per-lane copy with a known byte count, used to calibrate
// rocprofv3's FETCH_SIZE / WRITE_SIZE for the access width the stage kernels use

__global__ void probe_copy_kernel(double* __restrict__ dst, const double* __restrict__ src, long n)
{
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x)
    dst[e] = src[e];
}

// ------------------------------------------------------------------------------------------
// slab object + shim

// a z-neighbour's buffers mapped into this process (ipc transport): the put kernel and the fused
// stage kernels store this slab's boundary planes straight into the neighbour's ghost plane
struct SlabPeer {
  int on;                              // 1: a neighbour on this side receives our boundary planes
  int opened;                          // 1: base[] / sig came from hipIpcOpenMemHandle (close them)
  double* base[PFT_BUF_COUNT];         // the neighbour's buffers by physical index
  unsigned long long* sig;             // the neighbour's flag words
  long fs;                             // its field stride
  int n3;                              // its interior planes
  int remote;                          // 1: on another GPU (xGMI)
  int staged;                          // 1: our planes go to its receive buffer (remote, or PFT_IPC_STAGED)
  double* rbuf;                        // its receive buffer
};

struct pft_slab {
  pft_slab_desc d;
  pft_consts c;
  long fs;
  int plane;
  double* buf[PFT_BUF_COUNT];
  double* buf0[PFT_BUF_COUNT];   // the allocations by physical index (buf[] is permuted by swaps)
  int phys[PFT_BUF_COUNT];       // role -> physical index; every rank swaps identically, so a role
                                 // names the same physical buffer on every slab
  unsigned long long* sig;       // flag words written by the neighbours: [0] from below, [1] from
                                 // above (monotonic exchange sequence numbers); [8] put counter
  double* rbuf;                  // staged receive buffer (uncached, 2 x 12 planes; pft_slab_ipc_export)
  // copy-engine puts (pft_slab_halo_put_ce): the flags are raised by 8-byte SDMA copies from this
  // device table of sequence numbers (seq_base + 1 .. seq_base + PFT_SEQTAB), refilled from the
  // pinned halves seqhost[] when an exchange's number leaves it
  unsigned long long* seqtab;
  unsigned long long* seqhost;
  unsigned long long seq_base;
  int seq_half, seq_n;
  hipEvent_t ev_seq[2];  // recorded after each refill's H2D copy from that pinned half: the host
                         // rewrites a half only once the copy that read it last has run
  // the flags behind the completed plane copies (pft_slab_halo_put_ce, ce_fence): an event after
  // each copy stream's planes, waited for by the OTHER copy stream, which raises that side's flag
  int ce_fence;
  int gpu_ranks;         // ranks of the communicator on this slab's GPU (ipc attach; 0/1: alone)
  hipEvent_t ev_planes[2];
  // boundary launches on their own stream (pft_slab_set_boundary_stream; the copy-engine exchange):
  // a launch of the boundary planes (PFT_K_BOUNDARY/2) runs on `bnd` beside the interior launch on
  // the compute stream instead of before it; the exchange waits for ev_bnd, and so does the compute
  // stream before the next launch (pft_slab_halo_wait).  bnd_mode 1: every boundary launch, 2: the
  // pair kernels' (run_pair), 3: the pair kernels', with the halo waits on `bnd` (the boundary pipeline)
  int bnd_mode, bnd_pending, ce_streams;
  int ce_marked;         // pft_slab_halo_mark recorded ev_order[0] after the launch the next put_ce sends
  int bnd_split;         // the exchange's boundary launch ran before its interior on the compute stream
  int wait_streamops;    // A/B: halo waits as hipStreamWaitValue64 (env PFT_WAIT_STREAMOPS=1)
  hipStream_t bnd;
  hipEvent_t ev_bnd, ev_pre, ev_copy, ev_side, ev_join;
  // bnd_mode 4 (inline boundary): the pair kernels' boundary chunks lead their interior launch
  // (PFT_K_INLINE); its boundary workgroups count themselves in *bdone, and the exchange's copies
  // wait behind bnd_trigger_kernel for the count bdone_target (inline_pending: not yet sent)
  unsigned long long* bdone;
  unsigned long long bdone_target;
  int inline_pending;
  int trig_early;        // A/B (PFT_CE_TRIG): 1 the trigger queued with the launch, 0 with the copies
  int stage_inline;      // A/B (PFT_CE_STAGE_INLINE): stage launches inline too (else boundary first)
  hipEvent_t ev_trig;
  int put_role, put_f0, put_f1, put_deep;   // the exchange the last halo_put2 sent (its wait receives it)
  SlabPeer peer[2];              // [0] the neighbour below, [1] above
  int drop_puts;                 // fault injection: halo puts and flag raises skipped (PFT_IPC_DROP_PUTS)
  int ipc_poisoned;              // an ipc wait timed out: the flag words were forced past every
                                 // sequence number, so no later halo wait would block -- every halo
                                 // exchange, wait and sync refuses (PFT_ERR_IPC_TIMEOUT) until
                                 // pft_slab_ipc_close resets the flags (a detach / re-attach);
                                 // 2: the watched communicator aborted (PFT_ERR_COMM_ABORTED, for good)
  double* staging;      // host padded layout on the device (for upload/download)
  long S;                // host padded block (one field)
  unsigned long long* scratch;  // [0] eps bits, [1] nonfinite flag
  unsigned long long* host_scratch;  // pinned
  unsigned long long* host_pub;      // pinned, coherent: written by publish_kernel
  unsigned long long* host_pub_dev;  // its device address
  hipStream_t stream, comm;
  hipStream_t side;      // error-norm read-back while the compute stream runs ahead
  hipEvent_t ev_order[3];  // stream-order events: [0] compute -> comm, [1] comm -> compute,
                           // [2] the last boundary launch on the comm stream
  hipEvent_t ev_eps;     // recorded on the compute stream after the error norm is final
  int eps_marked;        // 1: publish kernel + event; 2: published by stage 5 itself (pub ring)
  // in-kernel publication (pft_slab_set_inkernel_publish): ring of 2-word slots in pinned,
  // coherent host memory, one per stage-5 launch; the host pre-sets a slot to the sentinel and
  // polls it after the launch
  int inkernel_pub;
  unsigned long long* pub_ring;      // host address (PFT_PUB_SLOTS x 2 words)
  unsigned long long* pub_ring_dev;  // its device address
  unsigned int* pub_count;           // device: finished workgroups of the publishing launch
  EpsShard* eps_shards;              // device: the error norm's shards (after pub_count's line)
  unsigned long long* part;          // device: deferred publication partials (2 words per workgroup)
  long part_cap;                     // ... their capacity in workgroups
  int defer_n;                       // workgroups of the armed error-norm launch awaiting reduction
  int defer_slot;                    // ... and its host slot
  int split_pub;                     // a split stage 4+5's boundary launch armed it; the interior follows
  // host-side memos (a small slab is host-bound: ~5 launches of a few us per attempted step)
  int fgeo_valid, fgeo_wx, fgeo_ty;  // fused_geometry(n1, n2) of this slab
  double fgeo_eff;
  long kz_key[16];                   // z-chunk cost model: key (occupancy, tiles, planes) -> kz
  int kz_val[16];
  long pub_next;                     // slots used so far
  int pub_armed;                     // the last stage-5 launch publishes into slot pub_slot
  int pub_slot;
  // gated steps (f4, pft_slab_gate_*): the host's decisions on the next step go to a ring of
  // pinned slots (4 words: seq, t bits, h bits, pad); the speculative stage 1's extra workgroup
  // copies its slot into the device ring, which the pre-enqueued launches of that step read
  unsigned long long* gate_pin;      // host address, PFT_GATE_SLOTS x 4 words
  unsigned long long* gate_pin_dev;  // its device address
  unsigned long long* gate_dev;      // device ring, PFT_GATE_SLOTS x 4 words
  unsigned long long gate_seq;       // the last sequence number handed out
  unsigned long long gate_arm_seq;   // the next speculative stage-1 launch decides this step ...
  double gate_arm_t, gate_arm_h;     // ... (t, h) of it (ignored when that launch is gated itself)
  unsigned long long gate_use_seq;   // launches enqueued now are gated on this decision (0: not)
  double gate_final, gate_delta, gate_hmin;   // the solve's constants (pft_slab_gate_config)
  int gate_local, gate_nan;
  int gate_flip;         // test hook, env PFT_GATE_FLIP (StageArgs::d_flip)
  // eps-publication bookkeeping snapshots (pft_slab_book_save/load): the launches of the next
  // step are enqueued between this step's launches and the read of its error norm
  struct Book {
    long pub_next;
    int pub_armed, pub_slot, eps_marked, defer_n, defer_slot;
  } book[2];
  int kz;                // planes per workgroup z-march; 0 = automatic (z-chunk cost model)
  int n_cu;               // compute units of the slab's device
  int cu_reserved;        // of them kept off the compute stream for the boundary launches (CU mask)
  double* noise;         // device u_noise (n3*plane) or null
  int tile_wx;           // 32 / 16: LDS-tiled kernels with that many pairs per row; 1: automatic;
                         // 2: LDS-tiled at any size, automatic tile; 0: cache-based
  int n1_tiled_ok;
  int recompute;         // 1: stage inputs rebuilt from x and the K's (no aux arrays)
  int gl_keep;           // X and XN hold the same gl, and x + c*0.0 == x for every gl value
  int pair_on;           // pair kernels (merson_pair): 0 off, 1 automatic (large slabs), 2 wherever
                         // they fit (pft_slab_set_pair); env PFT_PAIR overrides
  int pair_env;          // PFT_PAIR was set
  int pair_tx, pair_ty;  // pair tile (pair_geometry, once per slab); 0 x 0: none fits
  long pair_ntile;
  double timeout_s;      // bound on a host wait for the compute stream while ipc peers are on
                         // (env PFT_IPC_TIMEOUT, default 300 s; slab_wait)
  pft_slab_watch_fn watch;   // communicator watchdog (RCCL: async error / expiry -> abort)
  void* watch_ctx;
  double watch_timeout_s;
  // per-stage timing: a ring of begin/end event pairs, so that kernels still running when the
  // host collects (the speculative stage 1) are picked up by a later collect
  hipEvent_t tev[6][PFT_TRING][2];
  int thead[6], ttail[6];      // next slot to record / oldest slot not yet collected
  double tacc_ms[6];           // collected but not yet handed out
  long tacc_n[6];
};

static double wall_s()
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

// A dead or diverged ipc peer never raises the flag word the compute stream waits on
// (hipStreamWaitValue64, pft_slab_halo_wait), so the stream would never drain.  On expiry of
// s->timeout_s the slab raises its own flag words past every sequence number (on the side stream,
// which nothing blocks): the compute stream drains -- its results are void -- and the caller gets
// PFT_ERR_IPC_TIMEOUT, which RK_MPI_SA_solve reports as PFT_SOLVE_DEVICE_ERROR.
static int slab_poisoned(pft_slab* s, const char* what)
{
  if (s->ipc_poisoned == 2) {
    snprintf(g_err, sizeof(g_err), "%s: the slab's communicator was aborted (PFT_COMM_TIMEOUT or an asynchronous error)", what);
    return PFT_ERR_COMM_ABORTED;
  }
  snprintf(g_err, sizeof(g_err), "%s: an earlier ipc halo wait timed out; detach and re-attach the slab", what);
  return PFT_ERR_IPC_TIMEOUT;
}

// the communicator watchdog (pft_slab_set_watch), called about every millisecond of a host wait;
// t0: when the wait began (0: not yet taken).  Nonzero: the communicator aborted -- the slab
// refuses from now on (its streams drained inside the abort, or will never: no later wait trusts them)
static int slab_watch(pft_slab* s, double* t0, const char* what)
{
  if (*t0 == 0.0) *t0 = wall_s();
  const int expired = wall_s() - *t0 > s->watch_timeout_s;
  const int rc = s->watch(s->watch_ctx, expired);
  if (!rc) return 0;
  s->ipc_poisoned = 2;
  snprintf(g_err, sizeof(g_err), "%s: the communicator aborted (%s)", what,
           expired ? "no progress within PFT_COMM_TIMEOUT" : "asynchronous error");
  fprintf(stderr, "libpft: %s\n", g_err);
  return rc;
}

static int slab_timed_out(pft_slab* s, const char* what)
{
  static const unsigned long long released[2] = {~0ULL >> 1, ~0ULL >> 1};
  s->ipc_poisoned = 1;
  // on a stream of its own: the slab's other streams may hold copies waiting (through events) for
  // the blocked compute stream (the copy-engine exchange)
  hipStream_t rel = nullptr;
  if (hipStreamCreateWithFlags(&rel, hipStreamNonBlocking) == hipSuccess) {
    (void)hipMemcpyAsync(s->sig, released, sizeof(released), hipMemcpyHostToDevice, rel);
    (void)hipStreamSynchronize(rel);
    (void)hipStreamDestroy(rel);
  }
  (void)hipStreamSynchronize(s->stream);
  (void)hipGetLastError();
  snprintf(g_err, sizeof(g_err), "%s: no halo from an ipc neighbour within %.0f s (PFT_IPC_TIMEOUT)", what,
           s->timeout_s);
  fprintf(stderr, "libpft: %s\n", g_err);
  return PFT_ERR_IPC_TIMEOUT;
}

// the host waits for an event (or the whole compute stream when ev is null): unbounded with no ipc
// peer, bounded by s->timeout_s with one
static int slab_wait(pft_slab* s, hipEvent_t ev, const char* what)
{
  if (s->ipc_poisoned) {
    // ipc: the released flags let the stream drain: wait for it, then refuse.  An aborted
    // communicator: refuse at once (nothing guarantees the stream drains)
    if (s->ipc_poisoned == 1) (void)hipStreamSynchronize(s->stream);
    (void)hipGetLastError();
    return slab_poisoned(s, what);
  }
  if (!ev && s->bnd_mode == 3 && s->bnd && s->ev_join) {
    // the boundary pipeline: a wait for the compute stream includes the boundary stream (its
    // halo waits and staged receives write ghost planes the host or the next call may read)
    HIPCHK(hipEventRecord(s->ev_join, s->bnd));
    HIPCHK(hipStreamWaitEvent(s->stream, s->ev_join, 0));
  }
  if (!s->peer[0].on && !s->peer[1].on && !s->watch) {
    HIPCHK(ev ? hipEventSynchronize(ev) : hipStreamSynchronize(s->stream));
    return 0;
  }
  const double t0 = wall_s();
  double tw = 0.0;
  for (long it = 0;; ++it) {
    const hipError_t q = ev ? hipEventQuery(ev) : hipStreamQuery(s->stream);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return fail(q, what);
    if (it < 20000) {
      __builtin_ia32_pause();
    } else {
      sched_yield();
      if ((it & 1023) == 0) {
        if (s->watch) {
          const int rc = slab_watch(s, &tw, what);
          if (rc) return rc;
        } else if (wall_s() - t0 > s->timeout_s) {
          return slab_timed_out(s, what);
        }
      }
    }
  }
}

extern "C" {

int pft_slab_sync(pft_slab* s) { return s ? slab_wait(s, nullptr, "pft_slab_sync") : -2; }

int pft_slab_set_watch(pft_slab* s, pft_slab_watch_fn fn, void* ctx, double timeout_s)
{
  if (!s || (fn && !(timeout_s > 0.0))) return -2;
  s->watch = fn;
  s->watch_ctx = fn ? ctx : nullptr;
  s->watch_timeout_s = timeout_s;
  return 0;
}

const char* pft_hip_last_error(void) { return g_err; }

int pft_hip_device_count(int* n)
{
  HIPCHK(hipGetDeviceCount(n));
  return 0;
}
int pft_hip_set_device(int dev)
{
  HIPCHK(hipSetDevice(dev));
  return 0;
}
int pft_hip_get_device(int* dev)
{
  HIPCHK(hipGetDevice(dev));
  return 0;
}

int pft_hip_device_phys_id(int dev, int* id)
{
  // the GPU's PCI location (domain, bus, device): the same physical GPU has the same id in every
  // process, whatever each process's device numbering (HIP_VISIBLE_DEVICES)
  int dom = 0, bus = 0, pdev = 0;
  HIPCHK(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, dev));
  HIPCHK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev));
  HIPCHK(hipDeviceGetAttribute(&pdev, hipDeviceAttributePciDeviceId, dev));
  *id = ((dom & 0xffff) << 13) | ((bus & 0xff) << 5) | (pdev & 0x1f);
  return 0;
}
int pft_hip_device_ident(int dev, char* buf, int len)
{
  if (!buf || len < PFT_DEV_IDENT_BYTES) return -2;
  char bus[32] = {0};
  hipUUID u;
  memset(&u, 0, sizeof(u));
  HIPCHK(hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, dev));
  HIPCHK(hipDeviceGetUuid(&u, dev));
  int n = snprintf(buf, (size_t)len, "%s/", bus);
  for (int i = 0; i < 16 && n < len - 2; ++i) n += snprintf(buf + n, (size_t)(len - n), "%02x", (unsigned char)u.bytes[i]);
  return 0;
}
int pft_hip_device_sync(void)
{
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

static long pair_geometry(int n1, int n2, int* tx_out, int* ty_out);

int pft_slab_create(pft_slab** out, const pft_slab_desc* d, const pft_consts* c)
{
  *out = nullptr;
  if (d->n1 < 1 || d->n2 < 1 || d->n3 < 1) return -2;
  pft_slab* s = new pft_slab();
  memset(s, 0, sizeof(*s));
  s->d = *d;
  s->c = *c;
  s->plane = d->n1 * d->n2;
  // a field: far ghost plane, ghost plane, n3 interior planes, ghost plane, far ghost plane; the
  // buffer pointer points at the first ghost plane (plane 0 of the kernels' indexing)
  const long raw = (long)(d->n3 + 4) * s->plane;
  s->fs = (raw + 63) & ~63L;  // 512-byte aligned field strides
  s->S = (long)(d->n1 + 4) * (d->n2 + 4) * (d->n3 + 4);
  s->kz = 0;
  s->tile_wx = 1;
  s->n1_tiled_ok = 1;
  s->recompute = 1;
  {
    // fault injection (tests/test_ipc_multiprocess.py): this slab never delivers its halo -- no
    // put, no flag raise -- as a peer that died would not
    const char* ed = getenv("PFT_IPC_DROP_PUTS");
    s->drop_puts = ed ? atoi(ed) : 0;
    // pair kernels where the slab qualifies (pft_slab_pair_ok); env PFT_PAIR=0 turns them off (A/B)
    const char* ep = getenv("PFT_PAIR");
    s->pair_env = ep != nullptr;
    s->pair_on = ep ? atoi(ep) : 1;
    s->pair_ntile = pair_geometry(d->n1, d->n2, &s->pair_tx, &s->pair_ty);
    const char* eg = getenv("PFT_GATE_FLIP");
    s->gate_flip = eg ? atoi(eg) : 0;
    const char* ew = getenv("PFT_WAIT_STREAMOPS");
    s->wait_streamops = ew ? atoi(ew) : 0;
    const char* et = getenv("PFT_IPC_TIMEOUT");
    s->timeout_s = (et && atof(et) > 0.0) ? atof(et) : 300.0;
  }
  const size_t bytes = sizeof(double) * (3 * (size_t)s->fs + 2 * (size_t)s->plane);
  hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  // the halo exchange's stream at the greatest priority: its RCCL kernel is dispatched ahead of
  // the interior sweep's workgroups when both become ready
  int prio_lo = 0, prio_hi = 0;
  if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&s->comm, hipStreamNonBlocking, prio_hi);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s->ev_eps, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s->ev_order[0], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s->ev_order[1], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s->ev_order[2], hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc((void**)&s->scratch, 64);
  if (e == hipSuccess) e = hipHostMalloc((void**)&s->host_scratch, 64, hipHostMallocDefault);
  if (e == hipSuccess) e = hipHostMalloc((void**)&s->host_pub, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->host_pub_dev, s->host_pub, 0);
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&s->pub_ring, 16 * PFT_PUB_SLOTS, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->pub_ring_dev, s->pub_ring, 0);
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&s->gate_pin, 32 * PFT_GATE_SLOTS, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->gate_pin_dev, s->gate_pin, 0);
  if (e == hipSuccess) memset(s->gate_pin, 0, 32 * PFT_GATE_SLOTS);
  if (e == hipSuccess) e = hipMalloc((void**)&s->gate_dev, 32 * PFT_GATE_SLOTS);
  if (e == hipSuccess) e = hipMemsetAsync(s->gate_dev, 0, 32 * PFT_GATE_SLOTS, s->stream);
  // two sets of error-norm shards: a boundary launch uses the second, so that it may run beside the
  // interior launch of the same stage (pft_slab_set_boundary_stream)
  const size_t cnt_bytes = 64 + sizeof(EpsShard) * 2 * PFT_EPS_SHARDS;
  if (e == hipSuccess) e = hipMalloc((void**)&s->pub_count, cnt_bytes);
  if (e == hipSuccess) e = hipMemsetAsync(s->pub_count, 0, cnt_bytes, s->stream);
  if (e == hipSuccess) s->eps_shards = (EpsShard*)((char*)s->pub_count + 64);
  // the flag words are polled by the command processor (hipStreamWaitValue64) and written by a
  // neighbour -- possibly another GPU over xGMI: uncached device memory, so that no cache between
  // the writer and the poller can hold a stale copy
  if (e == hipSuccess) e = hipExtMallocWithFlags((void**)&s->sig, 4096, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemsetAsync(s->sig, 0, 4096, s->stream);
  for (int b = 0; b < PFT_BUF_COUNT && e == hipSuccess; ++b) {
    e = hipMalloc((void**)&s->buf0[b], bytes);
    s->buf[b] = s->buf0[b] + s->plane;   // past the first field's far ghost plane
    s->phys[b] = b;
    // zero-fill on the slab's own stream: the compute stream is non-blocking, so a fill on the
    // null stream would not be ordered before the first upload/kernel (it raced with them)
    if (e == hipSuccess) e = hipMemsetAsync(s->buf0[b], 0, bytes, s->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  int dev = 0;
  if (e == hipSuccess) e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&s->n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) {
    pft_slab_destroy(s);
    return fail(e, "slab buffers/streams");
  }
  *out = s;
  return 0;
}

int pft_slab_destroy(pft_slab* s)
{
  if (!s) return 0;
  (void)pft_slab_ipc_close(s);
  for (int b = 0; b < PFT_BUF_COUNT; ++b)
    if (s->buf0[b]) (void)hipFree(s->buf0[b]);
  if (s->sig) (void)hipFree(s->sig);
  if (s->rbuf) (void)hipFree(s->rbuf);
  if (s->seqtab) (void)hipFree(s->seqtab);
  if (s->seqhost) (void)hipHostFree(s->seqhost);
  if (s->staging) (void)hipFree(s->staging);
  if (s->noise) (void)hipFree(s->noise);
  for (int st = 0; st < 6; ++st)
    for (int e = 0; e < 2; ++e)
      for (int r = 0; r < PFT_TRING; ++r)
        if (s->tev[st][r][e]) (void)hipEventDestroy(s->tev[st][r][e]);
  if (s->scratch) (void)hipFree(s->scratch);
  if (s->host_scratch) (void)hipHostFree(s->host_scratch);
  if (s->host_pub) (void)hipHostFree(s->host_pub);
  if (s->pub_ring) (void)hipHostFree(s->pub_ring);
  if (s->gate_pin) (void)hipHostFree(s->gate_pin);
  if (s->gate_dev) (void)hipFree(s->gate_dev);
  if (s->pub_count) (void)hipFree(s->pub_count);
  if (s->part) (void)hipFree(s->part);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  if (s->comm) (void)hipStreamDestroy(s->comm);
  if (s->side) (void)hipStreamDestroy(s->side);
  if (s->bnd) (void)hipStreamDestroy(s->bnd);
  if (s->ev_bnd) (void)hipEventDestroy(s->ev_bnd);
  if (s->ev_pre) (void)hipEventDestroy(s->ev_pre);
  if (s->ev_copy) (void)hipEventDestroy(s->ev_copy);
  if (s->ev_side) (void)hipEventDestroy(s->ev_side);
  if (s->ev_join) (void)hipEventDestroy(s->ev_join);
  if (s->ev_trig) (void)hipEventDestroy(s->ev_trig);
  if (s->bdone) (void)hipFree(s->bdone);
  for (int i = 0; i < 2; ++i) {
    if (s->ev_seq[i]) (void)hipEventDestroy(s->ev_seq[i]);
    if (s->ev_planes[i]) (void)hipEventDestroy(s->ev_planes[i]);
  }

  if (s->ev_eps) (void)hipEventDestroy(s->ev_eps);
  for (int i = 0; i < 3; ++i)
    if (s->ev_order[i]) (void)hipEventDestroy(s->ev_order[i]);
  delete s;
  return 0;
}

size_t pft_slab_state_bytes(const pft_slab* s) { return sizeof(double) * 3 * (size_t)s->fs; }
void* pft_slab_stream(pft_slab* s) { return (void*)s->stream; }
void* pft_slab_comm_stream(pft_slab* s) { return (void*)s->comm; }
double* pft_slab_buffer(pft_slab* s, int which) { return (which >= 0 && which < PFT_BUF_COUNT) ? s->buf[which] : nullptr; }
size_t pft_slab_field_stride(const pft_slab* s) { return (size_t)s->fs; }
size_t pft_slab_plane(const pft_slab* s) { return (size_t)s->plane; }
int pft_slab_nz(const pft_slab* s) { return s->d.n3; }
void* pft_slab_scratch(pft_slab* s) { return (void*)s->scratch; }
const pft_slab_desc* pft_slab_get_desc(const pft_slab* s) { return &s->d; }
int pft_slab_set_tile(pft_slab* s, int wx)
{
  if (wx != 0 && wx != 1 && wx != 2 && wx != 16 && wx != 32) return -2;
  s->tile_wx = wx;
  return 0;
}

int pft_slab_set_kz(pft_slab* s, int kz)
{
  if (kz < 0) return -2;
  s->kz = kz;
  return 0;
}

static int ensure_staging(pft_slab* s)
{
  if (s->staging) return 0;
  HIPCHK(hipMalloc((void**)&s->staging, sizeof(double) * 3 * (size_t)s->S));
  return 0;
}

int pft_slab_upload_host(pft_slab* s, int which, const double* host_padded)
{
  // X and XN may differ now: the caller re-establishes it (an upload of a stage buffer, e.g. A0
  // for a host-side RHS evaluation, leaves it alone)
  if (which == PFT_BUF_X || which == PFT_BUF_XN) s->gl_keep = 0;
  int rc = ensure_staging(s);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(s->staging, host_padded, sizeof(double) * 3 * (size_t)s->S, hipMemcpyHostToDevice,
                        s->stream));
  pack_kernel<<<2048, 256, 0, s->stream>>>(s->staging, s->buf[which], s->d.n1, s->d.n2, s->d.n3, s->fs, s->S);
  HIPCHK(hipGetLastError());
  return slab_wait(s, nullptr, "upload");
}

int pft_slab_download_host(pft_slab* s, int which, double* host_padded)
{
  int rc = ensure_staging(s);
  if (rc) return rc;
  // staging keeps the host's ghost values (copied in first), interior overwritten
  HIPCHK(hipMemcpyAsync(s->staging, host_padded, sizeof(double) * 3 * (size_t)s->S, hipMemcpyHostToDevice,
                        s->stream));
  unpack_kernel<<<2048, 256, 0, s->stream>>>(s->buf[which], s->staging, s->d.n1, s->d.n2, s->d.n3, s->fs, s->S);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(host_padded, s->staging, sizeof(double) * 3 * (size_t)s->S, hipMemcpyDeviceToHost,
                        s->stream));
  return slab_wait(s, nullptr, "download");
}

}  // extern "C"

// kernel flavours: KCACHE (any n1, aux arrays), KFUSED (LDS tile, stage inputs recomputed from x
// and the K's -- the default for even n1); 1 was the retired LDS-tiled aux-array kernel
enum { KCACHE = 0, KFUSED = 2 };

// resident workgroups per CU of the kernel launch_kernel would run (hipOccupancy..., cached)
template <int STAGE, int MODE, bool GLS>
static int kernel_occupancy(int kind, int wx)
{
  static int cache[3] = {0, 0, 0};
  (void)wx;
  int& n = cache[kind];
  if (n) return n;
  const void* f = kind == KFUSED ? (const void*)merson_fused<STAGE, MODE, GLS>
                                 : (const void*)merson_stage<STAGE, MODE, GLS>;
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, kind == KFUSED ? PFT_FBLOCK : PFT_BLOCK, 0) != hipSuccess || b < 1) b = 1;
  n = b;
  return n;
}

template <int STAGE, bool GLS>
static int occupancy_mode(int mode, int kind, int wx)
{
  switch (mode) {
    case 0: return kernel_occupancy<STAGE, 0, GLS>(kind, wx);
    case 1: return kernel_occupancy<STAGE, 1, GLS>(kind, wx);
    case 2: return kernel_occupancy<STAGE, 2, GLS>(kind, wx);
    case 10: return kernel_occupancy<STAGE, 10, GLS>(kind, wx);
    default: return kernel_occupancy<STAGE, 11, GLS>(kind, wx);
  }
}

static int stage_occupancy(int stage, int mode, int gls, int kind, int wx)
{
  switch (stage) {
    case 0: return gls ? occupancy_mode<0, true>(mode, kind, wx) : occupancy_mode<0, false>(mode, kind, wx);
    case 1: return gls ? occupancy_mode<1, true>(mode, kind, wx) : occupancy_mode<1, false>(mode, kind, wx);
    case 2: return gls ? occupancy_mode<2, true>(mode, kind, wx) : occupancy_mode<2, false>(mode, kind, wx);
    case 3: return gls ? occupancy_mode<3, true>(mode, kind, wx) : occupancy_mode<3, false>(mode, kind, wx);
    case 4: return gls ? occupancy_mode<4, true>(mode, kind, wx) : occupancy_mode<4, false>(mode, kind, wx);
    default: return gls ? occupancy_mode<5, true>(mode, kind, wx) : occupancy_mode<5, false>(mode, kind, wx);
  }
}

template <int STAGE, int MODE, bool GLS>
static void launch_kernel(int kind, int wx, dim3 g, hipStream_t st, const StageArgs& a, const pft_consts& c)
{
  if (kind == KFUSED) {
    merson_fused<STAGE, MODE, GLS><<<g, PFT_FBLOCK, 0, st>>>(a, c);
  } else {
    merson_stage<STAGE, MODE, GLS><<<g, PFT_BLOCK, 0, st>>>(a, c);
  }
}

template <int STAGE, bool GLS>
static void launch_mode(int mode, int kind, int wx, dim3 g, hipStream_t st, const StageArgs& a,
                        const pft_consts& c)
{
  switch (mode) {
    case 0: launch_kernel<STAGE, 0, GLS>(kind, wx, g, st, a, c); break;
    case 1: launch_kernel<STAGE, 1, GLS>(kind, wx, g, st, a, c); break;
    case 2: launch_kernel<STAGE, 2, GLS>(kind, wx, g, st, a, c); break;
    case 10: launch_kernel<STAGE, 10, GLS>(kind, wx, g, st, a, c); break;
    case 11: launch_kernel<STAGE, 11, GLS>(kind, wx, g, st, a, c); break;
  }
}

template <bool GLS>
static void launch_stage(int stage, int mode, int kind, int wx, dim3 g, hipStream_t st, const StageArgs& a,
                         const pft_consts& c)
{
  switch (stage) {
    case 0: launch_mode<0, GLS>(mode, kind, wx, g, st, a, c); break;
    case 1: launch_mode<1, GLS>(mode, kind, wx, g, st, a, c); break;
    case 2: launch_mode<2, GLS>(mode, kind, wx, g, st, a, c); break;
    case 3: launch_mode<3, GLS>(mode, kind, wx, g, st, a, c); break;
    case 4: launch_mode<4, GLS>(mode, kind, wx, g, st, a, c); break;
    case 5: launch_mode<5, GLS>(mode, kind, wx, g, st, a, c); break;
  }
}

extern "C" {

// merson_fused tile: wx cell pairs x ty rows, 256 threads.  Limits: wx * ty <= 256 threads, the
// halo ring (2 wx + 4 + 2 ty pairs per field, 3 fields) loaded by one pass of the 256 threads,
// (2 wx + 4)(ty + 2) <= PFT_FUSED_LF doubles of LDS per field and plane.
static bool fused_geometry_ok(int wx, int ty)
{
  return wx >= 4 && ty >= 1 && wx * ty <= PFT_FBLOCK && 3 * (2 * wx + 4 + 2 * ty) <= PFT_FBLOCK &&
         (2 * wx + 4) * (ty + 2) <= PFT_FUSED_LF;
}

// automatic choice: 16..40 pairs wide (rows of 256-640 B), the tallest rows count that fits, and
// of those the tile whose workgroups carry the fewest idle lanes over the whole plane (edge tiles,
// threads beyond wx * ty); within 0.5% the wider.  Measured: with 64 x 8 tiles at n1 = 200 a
// quarter of the workgroups are 7/8 idle; a z-march of 64-wide tiles streams at 4.7-4.9 TB/s
// there and at 5.2-5.4 TB/s when n1 is a multiple of 64 (scripts/probes/stream_probe.hip).
// n1 = 200 and 400: 25 x 10 pairs (50 x 10 cells), all lanes but 6 busy.
static double fused_geometry(int n1, int n2, int* wx_out, int* ty_out)
{
  const int np = n1 / 2;
  double best = -1.0;
  int bw = 32, bt = 8;
  for (int wx = 16; wx <= 40; ++wx) {
    int ty = PFT_FBLOCK / wx;
    while (ty > 1 && !fused_geometry_ok(wx, ty)) --ty;
    if (!fused_geometry_ok(wx, ty)) continue;
    const long lanes = (long)((np + wx - 1) / wx) * ((n2 + ty - 1) / ty) * PFT_FBLOCK;
    const double eff = (double)np * n2 / (double)lanes;
    if (eff >= best - 0.005) {
      if (eff > best) best = eff;
      bw = wx;
      bt = ty;
    }
  }
  *wx_out = bw;
  *ty_out = bt;
  return best;   // busy lanes / launched lanes over the plane
}

// fused_geometry of the slab's plane, computed once (slab_kind and every launch ask for it)
static double slab_fgeo(const pft_slab* cs, int* wx, int* ty)
{
  pft_slab* s = const_cast<pft_slab*>(cs);
  if (!s->fgeo_valid) {
    s->fgeo_eff = fused_geometry(s->d.n1, s->d.n2, &s->fgeo_wx, &s->fgeo_ty);
    s->fgeo_valid = 1;
  }
  *wx = s->fgeo_wx;
  *ty = s->fgeo_ty;
  return s->fgeo_eff;
}

// z-chunk count memo: the cost models below scan every chunk count (400 planes: 400 candidates);
// their result only depends on the occupancy, the tile count and the planes
static int kz_memo_get(const pft_slab* s, int slot, long key)
{
  return s->kz_key[slot] == key + 1 ? s->kz_val[slot] : 0;
}
static void kz_memo_put(pft_slab* s, int slot, long key, int kz)
{
  s->kz_key[slot] = key + 1;
  s->kz_val[slot] = kz;
}

// planes per z-chunk: a CU runs `occ` workgroups at a time; a chunk count with w = ceil(workgroups /
// CUs) workgroups per CU costs (planes per chunk + the two planes a chunk re-reads) times
//   - occ <= 2: ceil(w / occ) rounds -- a partial last round runs a CU at half its waves and the
//     HBM-bound stages stall;
//   - occ >= 3: max(1, w / occ) -- retiring workgroups are refilled at once, and the extra
//     workgroups help the arithmetic-heavy stages hide latency.
// The cheapest count wins (more chunks only when 5% cheaper).
static int chunk_kz(pft_slab* s, int slot, int occ, long ntile, int nplanes, int min_nch = 1)
{
  const long key = ((long)occ << 52) ^ ((long)s->cu_reserved << 44) ^ (ntile << 24) ^ (long)nplanes;
  int kz = kz_memo_get(s, slot, key);
  if (kz) return kz;
  int best_nch = 1;
  double best_cost = -1.0;
  if (min_nch > nplanes) min_nch = nplanes;
  for (int nch = min_nch; nch <= nplanes; ++nch) {
    const int k = (nplanes + nch - 1) / nch;
    if (nch > min_nch && k == (nplanes + nch - 2) / (nch - 1)) continue;   // same kz as nch - 1
    if ((nplanes + k - 1) / k < min_nch) continue;
    if (min_nch >= 3 && (k < 2 || nplanes - ((nplanes + k - 1) / k - 1) * k < 2)) continue;   // edge chunks >= 2 planes
    const long nb = ntile * ((nplanes + k - 1) / k);
    const int ncu = s->n_cu - s->cu_reserved;   // the compute stream's CUs (launches on it chunk here)
    const long per_cu = (nb + ncu - 1) / ncu;
    const double rounds = occ <= 2 ? (double)((per_cu + occ - 1) / occ) : std::max(1.0, (double)per_cu / occ);
    const double cost = rounds * (k + 2);
    if (best_cost < 0.0 || cost < 0.95 * best_cost) { best_cost = cost; best_nch = nch; }
  }
  if (best_cost < 0.0) best_nch = std::max(1, nplanes);
  kz = (nplanes + best_nch - 1) / best_nch;
  kz_memo_put(s, slot, key, kz);
  return kz;
}

static int slab_kind(const pft_slab* s)
{
  // 16-byte rows need n1 even; the aux-array path (recompute off) is the cache kernel's.  (An
  // LDS-tiled aux-array kernel, 72 doubles per cell-step, was removed: measured slower than the
  // recompute kernel everywhere)
  if (s->d.n1 % 2 != 0 || s->tile_wx == 0 || !s->recompute) return KCACHE;
  // automatic choice: the LDS-tiled kernel unless its tiles leave most lanes idle (planes
  // narrower than a tile, e.g. n1 < 32); the cache kernel's flat 256-cell workgroups fit any
  // plane.  Measured at 100^3 (50 x 50 x 100, 25 x 10-pair tiles fit exactly): 4 810 vs 3 980
  // Mcells*steps/s (47 vs 60 us per attempted step untimed)
  if (s->tile_wx == 1) {
    int wx, ty;
    if (slab_fgeo(s, &wx, &ty) < 0.7) return KCACHE;
  }
  return KFUSED;
}

int pft_slab_stage_output(const pft_slab* s, int stage)
{
  // the buffer each stage of the step writes (and whose boundary planes neighbours need)
  static const int aux_out[6] = {-1, PFT_BUF_A0, PFT_BUF_A1, PFT_BUF_A0, PFT_BUF_A1, PFT_BUF_XN};
  static const int rc_out[6] = {-1, PFT_BUF_K1, PFT_BUF_A0 /* K2 */, PFT_BUF_K3, PFT_BUF_K4, PFT_BUF_XN};
  if (stage < 1 || stage > 5) return -2;
  return slab_kind(s) == KFUSED ? rc_out[stage] : aux_out[stage];
}

int pft_slab_tile_geometry(const pft_slab* s, int stage, int* wx, int* ty)
{
  const int kind = slab_kind(s);
  const bool auto_tile = s->tile_wx == 1 || s->tile_wx == 2;
  if (kind == KCACHE) {
    *wx = 0;
    *ty = 0;
  } else if (kind == KFUSED && auto_tile) {
    slab_fgeo(s, wx, ty);
  } else {
    *wx = s->tile_wx;
    *ty = PFT_FBLOCK / *wx;
  }
  return kind;
}

int pft_slab_stage_fields(const pft_slab* s, int stage)
{
  // fields of a stage's output buffer that the stage writes (stage 6: the speculative stage 1):
  // gl is not evolved under gl_static, and its K's are literal zeros on the recompute path
  if (stage < 1 || stage > 6) return -2;
  if (s->d.gl_static) return 2;
  if (slab_kind(s) == KFUSED && stage != 5) return 2;
  // stage 5 with gl_keep (agreed by every rank, rk_solver.c): gl's x(t+h) is not stored; the
  // neighbours' XN gl ghost planes already equal X's (both exchanged at upload)
  if (stage == 5 && pft_slab_get_gl_keep(s) && slab_kind(s) == KFUSED) return 2;
  return 3;
}

// arm the deferred publication of an error-norm launch of nwg workgroups into host slot j: its
// workgroups store partials (eps_store_part), the next stage-1 launch reduces and publishes them
static int defer_arm(pft_slab* s, long nwg, int j, unsigned long long** part, long cap_nwg = 0)
{
  if (std::max(nwg, cap_nwg) > s->part_cap) {
    if (s->part) HIPCHK(hipFree(s->part));
    s->part = nullptr;
    s->part_cap = 0;
    const long cap = std::max(std::max(nwg, cap_nwg), 4096L);
    HIPCHK(hipMalloc((void**)&s->part, 16 * (size_t)cap));
    s->part_cap = cap;
  }
  s->defer_n = (int)nwg;
  s->defer_slot = j;
  *part = s->part;
  return 0;
}

static int run_stage(pft_slab* s, int stage, const double* in, double* kout, double* out, double t_stage,
                     double coef, double h, int k_begin, int k_end, int gls, int kind)
{
  const int mode = s->d.calc_mode;
  if (mode != 0 && mode != 1 && mode != 2 && mode != 10 && mode != 11) return -2;
  // k_begin == PFT_K_BOUNDARY: the slab's two boundary planes (0 and n3 - 1) in ONE launch, two
  // one-plane chunks n3 - 1 planes apart (what the z-neighbours need first)
  const bool bnd = k_begin == PFT_K_BOUNDARY || k_begin == PFT_K_BOUNDARY2;
  const int bdepth = k_begin == PFT_K_BOUNDARY2 ? 2 : 1;   // PFT_K_BOUNDARY2: planes 0, 1 and n3-2, n3-1
  // inline boundary (merson_fused only, never gated): PFT_K_ENDS_FIRST -- the whole slab, the first
  // and last chunk of every tile column leading -- or PFT_K_INLINE -- two-plane chunks at each end
  // leading the interior [2, n3 - 2); ENDS_FIRST falls back to INLINE where the chunks cannot hold
  // the two planes at each end
  bool ends = k_begin == PFT_K_ENDS_FIRST;
  const bool inl = k_begin == PFT_K_INLINE || ends;
  if (inl && (kind != KFUSED || !s->bdone || s->d.n3 < 5 || s->gate_use_seq)) return -2;
  if (bnd || inl) {
    k_begin = 0;   // (inline: the planes are set below, once the chunking is known)
    k_end = s->d.n3;
  }
  if (k_begin < 0) k_begin = 0;
  if (k_end < 0 || k_end > s->d.n3) k_end = s->d.n3;
  if (k_end <= k_begin) return 0;
  StageArgs a;
  memset(&a, 0, sizeof(a));
  a.in = in;
  a.x = s->buf[PFT_BUF_X];
  a.k1 = s->buf[PFT_BUF_K1];
  a.k2 = s->buf[PFT_BUF_A0];
  a.k3 = s->buf[PFT_BUF_K3];
  a.k4 = s->buf[PFT_BUF_K4];
  a.kout = kout;
  a.out = out;
  a.noise = s->noise;
  a.eps_bits = s->scratch;
  a.shards = s->eps_shards + (bnd ? PFT_EPS_SHARDS : 0);
  a.nonfinite = (unsigned int*)(s->scratch + 1);
  a.fs = s->fs;
  a.n1 = s->d.n1;
  a.n2 = s->d.n2;
  a.n3 = s->d.n3;
  a.plane = s->plane;
  a.has_below = s->d.has_below;
  a.has_above = s->d.has_above;
  a.k_begin = k_begin;
  a.k_end = k_end;
  // tile width: 1 = per stage (measured at 400^3: the VALU-bound stages 0-2 run faster on 32x16
  // tiles -- fewer idle lanes at the x edge, 200 = 6.25 x 32 -- the HBM-bound stages 3-5 on 64x8)
  const bool auto_tile = s->tile_wx == 1 || s->tile_wx == 2;
  const int wx = kind == KCACHE ? 0 : auto_tile ? (stage <= 2 ? 16 : 32) : s->tile_wx;
  if (kind == KFUSED) {
    if (auto_tile) {
      slab_fgeo(s, &a.gwx, &a.gty);
    } else {
      a.gwx = s->tile_wx;
      a.gty = PFT_FBLOCK / s->tile_wx;
    }
    if (!fused_geometry_ok(a.gwx, a.gty)) return -2;
    a.ntile = ((s->d.n1 + 2 * a.gwx - 1) / (2 * a.gwx)) * ((s->d.n2 + a.gty - 1) / a.gty);
  } else if (wx) {
    const int TX = 2 * wx, TY = PFT_BLOCK / wx;
    a.ntile = ((s->d.n1 + TX - 1) / TX) * ((s->d.n2 + TY - 1) / TY);
  } else {
    a.ntile = (s->plane + PFT_BLOCK - 1) / PFT_BLOCK;
  }
  if (ends) {
    const int n3 = s->d.n3;
    const int occ = stage_occupancy(stage, mode, gls, kind, wx);
    const int kz = s->kz > 0 ? s->kz : chunk_kz(s, 14, occ, a.ntile, n3, 3);
    const int nch = (n3 + kz - 1) / kz;
    if (kz < 2 || nch < 3 || n3 - (nch - 1) * kz < 2) ends = false;
  }
  if (inl) {
    k_begin = ends ? 0 : 2;
    k_end = ends ? s->d.n3 : s->d.n3 - 2;
    a.k_begin = k_begin;
    a.k_end = k_end;
  }
  const int nplanes = k_end - k_begin;
  if (s->kz > 0) {
    a.kz = s->kz;
  } else if (ends) {
    a.kz = chunk_kz(s, 14, stage_occupancy(stage, mode, gls, kind, wx), a.ntile, nplanes, 3);
  } else {
    // automatic (chunk_kz)
    // Measured at 400^3 (80 tiles):
    // stage 5 (occ 2) 6 chunks, 0.348 ms vs 0.393 for 16; stage 1 (occ 3) 16 chunks of 25 planes,
    // 0.153 vs 0.163 for 9 of 45.  On a 400 x 400 x 100 slab (320 tiles, one 800^3 8-way rank)
    // stages 4-5: 3 chunks (960 workgroups, 2 rounds) 0.261 / 0.349 ms against 0.314 / 0.436 for
    // one round of 320 (64 CUs with 2 workgroups, 192 with 1).
    const int occ = stage_occupancy(stage, mode, gls, kind, wx);
    a.kz = chunk_kz(s, stage + 6 * (gls ? 1 : 0), occ, a.ntile, nplanes);
  }
  a.nchunk = (nplanes + a.kz - 1) / a.kz;
  a.kspan = a.kz;
  if (bnd) {
    a.kz = std::max(1, s->d.n3 - bdepth);
    a.kspan = bdepth;
    a.nchunk = s->d.n3 > bdepth ? 2 : 1;
  }
  a.nint = a.ntile * a.nchunk;
  if (inl) {
    a.bdone = s->bdone;
    if (ends) {
      const int nb = std::min(a.nchunk, 2);
      a.nbw = nb * a.ntile;
      a.bends = 1;
      a.c0 = 1;
      a.nint = (a.nchunk - nb) * a.ntile;
    } else {
      a.nbw = 2 * a.ntile;
    }
  }
  a.T_top = t_stage < s->c.phase_switch_time ? s->c.top_temp1 : s->c.top_temp2;
  a.coef = coef;
  a.h = h;
  // stage-input coefficients of the recompute path: exactly the solver's h/3.0, h/6.0, h/8.0, h
  a.cin = stage == 2 ? h / 3.0 : stage == 3 ? h / 6.0 : stage == 4 ? h / 8.0 : h;
  if (kind == KFUSED && in) a.x = in;    // pure RHS / speculative stage 1: the input is the given buffer
  // gl's x(t+h) is x + coef*(0.5*(0.0 + 0.0) + 2.0*0.0) (gl's K's are literal zeros): equal to x
  // bit for bit when coef is finite and no gl value is -0.0 or NaN, which the solver checked at
  // upload (pft_slab_set_gl_keep); XN's gl then already holds it, and stage 5 skips that store
  a.gl_keep = stage == 5 && kind == KFUSED && out && s->gl_keep && std::isfinite(coef) ? 1 : 0;
  if (kind == KFUSED && s->gate_use_seq) {
    // gated (pft_slab_gate_use): the scalars above are the launch's own (gate_scalars), from the
    // decision the host has not taken yet; the kernel ANDs isfinite(coef) into gl_keep
    const int j = (int)(s->gate_use_seq % PFT_GATE_SLOTS);
    a.gate = s->gate_dev + 4 * j;
    a.gseq = s->gate_use_seq;
    a.gl_keep = stage == 5 && out && s->gl_keep ? 1 : 0;
  }
  a.em0 = s->d.eps_mult[0];
  a.em1 = s->d.eps_mult[1];
  a.em2 = s->d.eps_mult[2];
  s->pub_armed = 0;
  if (stage == 5 && kind == KFUSED && out && !bnd && k_begin == 0 && k_end == s->d.n3 && s->inkernel_pub) {
    // the whole slab in one launch: its last workgroup publishes the error norm (slot pre-set to
    // the sentinel here, before the launch; the host polls it in pft_slab_eps_fetch)
    const int j = (int)(s->pub_next % PFT_PUB_SLOTS);
    __atomic_store_n(&s->pub_ring[2 * j], PFT_PUB_SENTINEL, __ATOMIC_RELEASE);
    __atomic_store_n(&s->pub_ring[2 * j + 1], PFT_PUB_SENTINEL, __ATOMIC_RELEASE);
    const int rc = defer_arm(s, (long)a.ntile * a.nchunk, j, &a.part);
    if (rc) return rc;
    s->pub_armed = 1;
    s->pub_slot = j;
  }
  dim3 g((unsigned)(a.nbw + a.nint));
  bool extra = false;
  // a stage launch's interior fills the chip: its boundary runs beside it only in bnd_mode 1 (slower:
  // the two launches' workgroups are dealt interleaved and the interior ends late).  In the boundary
  // pipeline (bnd_mode 3) the halo waits are on the boundary stream: a stage launch's boundary on
  // the compute stream first joins it
  const bool beside = bnd && s->bnd_mode == 1;
  if (bnd && s->bnd_mode == 3 && s->bnd) {
    HIPCHK(hipEventRecord(s->ev_join, s->bnd));
    HIPCHK(hipStreamWaitEvent(s->stream, s->ev_join, 0));
  }
  if (stage == 1 && kind == KFUSED && s->defer_n > 0) {
    // the previous error-norm launch's partials: reduced and published by one extra workgroup
    a.part = s->part;
    a.npart = s->defer_n;
    a.pub = s->pub_ring_dev + 2 * s->defer_slot;
    s->defer_n = 0;
    extra = true;
  }
  if (stage == 1 && kind == KFUSED && s->gate_arm_seq && in) {
    // the speculative stage 1 armed by pft_slab_gate_arm: its extra workgroup also decides the
    // step that just ended, for the next step's pre-enqueued launches and for the host
    const int j = (int)(s->gate_arm_seq % PFT_GATE_SLOTS);
    a.gpin = s->gate_pin_dev + 4 * j;
    a.gdev = s->gate_dev + 4 * j;
    a.gdec_seq = s->gate_arm_seq;
    a.dt = s->gate_arm_t;
    a.dh = s->gate_arm_h;
    a.d_final = s->gate_final;
    a.d_delta = s->gate_delta;
    a.d_hmin = s->gate_hmin;
    a.d_local = s->gate_local;
    a.d_nan = s->gate_nan;
    a.d_flip = s->gate_flip;
    __atomic_store_n(&s->gate_pin[4 * j], 0ULL, __ATOMIC_RELEASE);   // no decision yet
    s->gate_arm_seq = 0;
    extra = true;
  }
  if (extra) g.x += 1;
  hipStream_t st = s->stream;
  if (beside) {
    HIPCHK(hipEventRecord(s->ev_pre, s->stream));
    HIPCHK(hipStreamWaitEvent(s->bnd, s->ev_pre, 0));
    st = s->bnd;
  }
  if (gls)
    launch_stage<true>(stage, mode, kind, wx, g, st, a, s->c);
  else
    launch_stage<false>(stage, mode, kind, wx, g, st, a, s->c);
  HIPCHK(hipGetLastError());
  if (beside) {
    HIPCHK(hipEventRecord(s->ev_bnd, s->bnd));
    s->bnd_pending = 1;
  } else if (bnd) {
    s->bnd_split = 1;   // a boundary launch before its interior on the compute stream
  }
  if (inl) {
    // as run_pair: the copies' trigger queued with the launch
    s->bdone_target += (unsigned long long)a.nbw;
    s->inline_pending = 1;
    if (s->trig_early) {
      bnd_trigger_kernel<<<1, 64, 0, s->comm>>>(s->bdone, s->bdone_target);
      HIPCHK(hipGetLastError());
    }
  }
  return 0;
}

int pft_slab_stage(pft_slab* s, int stage, double t_stage, double coef, double h, int k_begin, int k_end)
{
  if (stage < 1 || stage > 5) return -2;
  const int kind = slab_kind(s);
  if (kind == KFUSED) {
    // inputs rebuilt from x, K1, K2 (in A0), K3, K4; outputs K_stage or x(t+h)
    static const int k_of[6] = {-1, PFT_BUF_K1, PFT_BUF_A0, PFT_BUF_K3, PFT_BUF_K4, -1};
    return run_stage(s, stage, nullptr, k_of[stage] >= 0 ? s->buf[k_of[stage]] : nullptr,
                     stage == 5 ? s->buf[PFT_BUF_XN] : nullptr, t_stage, coef, h, k_begin, k_end,
                     s->d.gl_static, kind);
  }
  // aux path: in -> (kout, out)
  static const int in_of[6] = {-1, PFT_BUF_X, PFT_BUF_A0, PFT_BUF_A1, PFT_BUF_A0, PFT_BUF_A1};
  static const int out_of[6] = {-1, PFT_BUF_A0, PFT_BUF_A1, PFT_BUF_A0, PFT_BUF_A1, PFT_BUF_XN};
  static const int k_of[6] = {-1, PFT_BUF_K1, -1, PFT_BUF_K3, PFT_BUF_K4, -1};
  return run_stage(s, stage, s->buf[in_of[stage]], k_of[stage] >= 0 ? s->buf[k_of[stage]] : nullptr,
                   s->buf[out_of[stage]], t_stage, coef, h, k_begin, k_end, s->d.gl_static, kind);
}

int pft_slab_rhs(pft_slab* s, int in_buf, int out_buf, double t)
{
  if (in_buf < 0 || in_buf >= PFT_BUF_COUNT || out_buf < 0 || out_buf >= PFT_BUF_COUNT) return -2;
  return run_stage(s, 0, s->buf[in_buf], s->buf[out_buf], nullptr, t, 0.0, 0.0, -1, -1, 0, slab_kind(s));
}

int pft_slab_set_gl_keep(pft_slab* s, int on)
{
  s->gl_keep = on ? 1 : 0;
  return 0;
}

int pft_slab_get_gl_keep(const pft_slab* s) { return s->gl_keep; }

int pft_slab_set_recompute(pft_slab* s, int on)
{
  s->recompute = on ? 1 : 0;
  return 0;
}

int pft_slab_set_consts(pft_slab* s, const pft_consts* c)
{
  s->c = *c;
  return 0;
}

int pft_slab_set_eps_mult(pft_slab* s, const double* em3)
{
  for (int q = 0; q < 3; ++q) s->d.eps_mult[q] = em3[q];
  return 0;
}

int pft_slab_set_noise(pft_slab* s, const double* host_noise)
{
  if (!host_noise) {
    if (s->noise) HIPCHK(hipFree(s->noise));
    s->noise = nullptr;
    return 0;
  }
  const size_t bytes = sizeof(double) * (size_t)s->plane * s->d.n3;
  if (!s->noise) HIPCHK(hipMalloc((void**)&s->noise, bytes));
  HIPCHK(hipMemcpy(s->noise, host_noise, bytes, hipMemcpyHostToDevice));
  return 0;
}

static int slab_ic_tables(pft_slab* s, const pft_ic_tables* t, int overlay, int* gl_unclean)
{
  if (!t || t->n1 != s->d.n1 || t->n2 != s->d.n2 || t->n3 != s->d.n3) return -2;
  const int n1 = t->n1, n2 = t->n2, n3 = t->n3, nb = t->nbeads;
  const long nbi = nb ? t->plane_off[n3] : 0;
  const size_t nd = 4 * (size_t)(n1 + n2 + n3) + 3 * (size_t)nb;
  const size_t ni = (size_t)(n3 + 1) + (size_t)nbi;
  std::vector<double> hd(nd);
  std::vector<int> hi(ni, 0);
  const double* src[12] = {t->tx1, t->tx2, t->px2, t->xb, t->ty1, t->ty2, t->py2, t->yb,
                           t->tz1, t->tz2, t->pz, t->zb};
  const int len[3] = {n1, n2, n3};
  size_t o = 0;
  for (int a = 0; a < 3; ++a)
    for (int q = 0; q < 4; ++q) {
      memcpy(&hd[o], src[4 * a + q], sizeof(double) * len[a]);
      o += len[a];
    }
  if (nb) {
    memcpy(&hd[o], t->bxyz, sizeof(double) * 3 * nb);
    memcpy(&hi[0], t->plane_off, sizeof(int) * (n3 + 1));
    if (nbi) memcpy(&hi[n3 + 1], t->plane_beads, sizeof(int) * nbi);
  }
  double* dd = nullptr;
  int* di = nullptr;
  unsigned int* du = nullptr;
  IcDev a;
  memset(&a, 0, sizeof(a));
  hipError_t e = hipMalloc((void**)&dd, sizeof(double) * nd);
  if (e == hipSuccess) e = hipMalloc((void**)&di, sizeof(int) * ni);
  if (e == hipSuccess) e = hipMalloc((void**)&du, sizeof(unsigned int));
  if (e == hipSuccess) e = hipMemcpyAsync(dd, hd.data(), sizeof(double) * nd, hipMemcpyHostToDevice, s->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(di, hi.data(), sizeof(int) * ni, hipMemcpyHostToDevice, s->stream);
  if (e == hipSuccess) e = hipMemsetAsync(du, 0, sizeof(unsigned int), s->stream);
  if (e == hipSuccess) {
    a.x = s->buf[PFT_BUF_X];
    a.xn = s->buf[PFT_BUF_XN];
    a.fs = s->fs;
    a.n1 = n1;
    a.n2 = n2;
    a.n3 = n3;
    a.plane = s->plane;
    a.tab = dd;
    a.poff = di;
    a.pbead = di + n3 + 1;
    a.nbeads = nb;
    a.u0 = t->u0;
    a.r2 = t->r2;
    a.s = t->s;
    a.R = t->R;
    a.reach2 = t->reach2;
    a.unclean = du;
    a.overlay = overlay;
    const long n = (long)s->plane * n3;
    ic_default_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s->stream>>>(a);
    e = hipGetLastError();
  }
  unsigned int hu = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&hu, du, sizeof(unsigned int), hipMemcpyDeviceToHost, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  (void)hipFree(dd);
  (void)hipFree(di);
  (void)hipFree(du);
  if (e != hipSuccess) return fail(e, "pft_slab_ic_default");
  if (gl_unclean) *gl_unclean = hu ? 1 : 0;
  return 0;
}

int pft_slab_ic_default(pft_slab* s, const pft_ic_tables* t, int* gl_unclean)
{
  return slab_ic_tables(s, t, 0, gl_unclean);
}

int pft_slab_ic_beads(pft_slab* s, const pft_ic_tables* t, int* gl_unclean)
{
  return slab_ic_tables(s, t, 1, gl_unclean);
}

int pft_slab_ic_program(pft_slab* s, int q, const pft_ic_prog* p, int clear)
{
  if (!p || q < 0 || q > 2 || p->n < 1) return -2;
  hipError_t e = hipSuccess;
  if (clear) {
    // the host array the reference's loop fills starts zeroed: quantities not yet initialised read 0
    e = hipMemsetAsync(s->buf[PFT_BUF_X], 0, sizeof(double) * 3 * (size_t)s->fs, s->stream);
    if (e == hipSuccess) e = hipMemsetAsync(s->buf[PFT_BUF_XN], 0, sizeof(double) * 3 * (size_t)s->fs, s->stream);
  }
  const size_t nt = (size_t)(p->ntab > 0 ? p->ntab : 1), nv = (size_t)(p->tab_len > 0 ? p->tab_len : 1);
  const size_t bytes = sizeof(int) * p->n + sizeof(double) * p->n + sizeof(int) * nt + sizeof(long) * nt +
                       sizeof(double) * nv + nv + 64;
  std::vector<char> h(bytes, 0);
  // one upload: [arg (n doubles)][tval (nv doubles)][toff (nt longs)][op (n ints)][taxis (nt ints)][terr]
  size_t o = 0;
  const size_t o_arg = o;  o += sizeof(double) * p->n;
  const size_t o_val = o;  o += sizeof(double) * nv;
  const size_t o_off = o;  o += sizeof(long) * nt;
  const size_t o_op = o;   o += sizeof(int) * p->n;
  const size_t o_ax = o;   o += sizeof(int) * nt;
  const size_t o_err = o;
  memcpy(&h[o_arg], p->arg, sizeof(double) * p->n);
  memcpy(&h[o_op], p->op, sizeof(int) * p->n);
  if (p->ntab > 0) {
    memcpy(&h[o_val], p->tab_val, sizeof(double) * p->tab_len);
    memcpy(&h[o_off], p->tab_off, sizeof(long) * p->ntab);
    memcpy(&h[o_ax], p->tab_axis, sizeof(int) * p->ntab);
    memcpy(&h[o_err], p->tab_err, p->tab_len);
  }
  char* d = nullptr;
  if (e == hipSuccess) e = hipMalloc((void**)&d, bytes);
  if (e == hipSuccess) e = hipMemcpyAsync(d, h.data(), bytes, hipMemcpyHostToDevice, s->stream);
  if (e == hipSuccess) {
    IcProgDev a;
    a.x = s->buf[PFT_BUF_X];
    a.xn = s->buf[PFT_BUF_XN];
    a.fs = s->fs;
    a.n1 = s->d.n1;
    a.n2 = s->d.n2;
    a.n3 = s->d.n3;
    a.plane = s->plane;
    a.q = q;
    a.n = p->n;
    a.arg = (const double*)(d + o_arg);
    a.tval = (const double*)(d + o_val);
    a.toff = (const long*)(d + o_off);
    a.op = (const int*)(d + o_op);
    a.taxis = (const int*)(d + o_ax);
    a.terr = (const unsigned char*)(d + o_err);
    const long n = (long)s->plane * s->d.n3;
    ic_prog_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s->stream>>>(a);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  if (d) (void)hipFree(d);
  if (e != hipSuccess) return fail(e, "pft_slab_ic_program");
  s->gl_keep = 0;
  return 0;
}

int pft_slab_order(pft_slab* s, int comm_first)
{
  // the second stream waits for the work enqueued so far on the first
  hipStream_t from = comm_first ? s->comm : s->stream, to = comm_first ? s->stream : s->comm;
  hipEvent_t ev = s->ev_order[comm_first ? 1 : 0];
  HIPCHK(hipEventRecord(ev, from));
  HIPCHK(hipStreamWaitEvent(to, ev, 0));
  return 0;
}

int pft_slab_eps_reset(pft_slab* s)
{
  HIPCHK(hipMemsetAsync(s->scratch, 0, 16, s->stream));
  return 0;
}

int pft_slab_eps_mark(pft_slab* s) { return pft_slab_eps_mark_on(s, (void*)s->stream); }

int pft_slab_set_inkernel_publish(pft_slab* s, int on)
{
  s->inkernel_pub = on ? 1 : 0;
  s->pub_armed = 0;
  s->split_pub = 0;
  s->defer_n = 0;
  return 0;
}

int pft_slab_eps_mark_on(pft_slab* s, void* stream)
{
  if (s->split_pub) {
    // a split stage 4+5 whose interior launch had no planes: the boundary's partials are all
    s->split_pub = 0;
    s->pub_armed = 1;
    s->pub_slot = s->defer_slot;
  }
  if (s->pub_armed && stream == (void*)s->stream) {
    // the stage-5 launch just enqueued publishes the error norm itself
    s->pub_armed = 0;
    s->pub_next++;
    s->eps_marked = 2;
    return 0;
  }
  // the error norm goes to coherent pinned host memory by a one-thread kernel (which also resets
  // it for the next step), and an event marks its completion: the host waits for that event
  // only, never for a copy queued behind (or beside) the speculative stage-1 kernel that follows
  // on the compute stream
  publish_kernel<<<1, 1, 0, (hipStream_t)stream>>>(s->scratch, s->host_pub_dev);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(s->ev_eps, (hipStream_t)stream));
  s->eps_marked = 1;
  return 0;
}

int pft_slab_eps_fetch(pft_slab* s, double* eps, int* nonfinite)
{
  if (s->ipc_poisoned) return slab_poisoned(s, "pft_slab_eps_fetch");
  if (s->eps_marked == 2) {
    // published beside the speculative stage 1 (deferred publication): poll the slot (pinned,
    // coherent) until both words left the sentinel while that kernel keeps running.  Without a
    // stage-1 launch since the error-norm launch, a one-workgroup reduction publishes instead.
    s->eps_marked = 0;
    if (s->defer_n > 0) {
      eps_reduce_kernel<<<1, 256, 0, s->stream>>>(s->part, s->defer_n, s->pub_ring_dev + 2 * s->defer_slot);
      s->defer_n = 0;
      HIPCHK(hipGetLastError());
    }
    volatile unsigned long long* w = s->pub_ring + 2 * s->pub_slot;
    long spins = 0;
    double t0 = 0.0;
    while (__atomic_load_n(&w[0], __ATOMIC_ACQUIRE) == PFT_PUB_SENTINEL ||
           __atomic_load_n(&w[1], __ATOMIC_ACQUIRE) == PFT_PUB_SENTINEL) {
      if (++spins < 200000) {
        __builtin_ia32_pause();
      } else if ((spins & 1023) == 0) {
        // long wait: make sure the stream is alive (a fault ends here with its error), and that an
        // ipc neighbour's halo has not been missing for longer than the slab's timeout
        const hipError_t q = hipStreamQuery(s->stream);
        if (q != hipSuccess && q != hipErrorNotReady) return fail(q, "hipStreamQuery (error norm poll)");
        if (q == hipSuccess && __atomic_load_n(&w[1], __ATOMIC_ACQUIRE) == PFT_PUB_SENTINEL)
          return fail(hipErrorUnknown, "error norm never published");
        if (s->watch) {
          const int rc = slab_watch(s, &t0, "error norm poll");
          if (rc) return rc;
        } else if (s->peer[0].on || s->peer[1].on) {
          if (t0 == 0.0) t0 = wall_s();
          else if (wall_s() - t0 > s->timeout_s) return slab_timed_out(s, "error norm poll");
        }
        sched_yield();
      }
    }
    s->host_scratch[0] = w[0];
    s->host_scratch[1] = w[1];
  } else if (s->eps_marked) {
    // read back on the side stream: work enqueued on the compute stream after the mark (the
    // speculative stage 1 of the next step) keeps running while the host decides
    s->eps_marked = 0;
    int rc = slab_wait(s, s->ev_eps, "error norm event");
    if (rc) return rc;
    s->host_scratch[0] = __atomic_load_n(&s->host_pub[0], __ATOMIC_ACQUIRE);
    s->host_scratch[1] = __atomic_load_n(&s->host_pub[1], __ATOMIC_ACQUIRE);
  } else {
    HIPCHK(hipMemcpyAsync(s->host_scratch, s->scratch, 16, hipMemcpyDeviceToHost, s->stream));
    int rc = slab_wait(s, nullptr, "error norm read-back");
    if (rc) return rc;
  }
  unsigned long long b = s->host_scratch[0];
  double v;
  memcpy(&v, &b, 8);
  *eps = v;
  if (nonfinite) *nonfinite = (int)(s->host_scratch[1] & 0xffffffffu);
  return 0;
}

static int timing_collect(pft_slab* s, bool wait)
{
  for (int st = 1; st <= 5; ++st) {
    while (s->ttail[st] < s->thead[st]) {
      hipEvent_t* ev = s->tev[st][s->ttail[st] % PFT_TRING];
      if (wait) {
        HIPCHK(hipEventSynchronize(ev[1]));
      } else {
        const hipError_t q = hipEventQuery(ev[1]);
        if (q == hipErrorNotReady) break;
        if (q != hipSuccess) return fail(q, "hipEventQuery");
      }
      float e = 0.f;
      HIPCHK(hipEventElapsedTime(&e, ev[0], ev[1]));
      s->tacc_ms[st] += (double)e;
      s->tacc_n[st] += 1;
      s->ttail[st]++;
    }
  }
  return 0;
}

static void timing_hand_out(pft_slab* s, double* ms, long* n)
{
  for (int st = 1; st <= 5; ++st) {
    ms[st] += s->tacc_ms[st];
    n[st] += s->tacc_n[st];
    s->tacc_ms[st] = 0.0;
    s->tacc_n[st] = 0;
  }
}

int pft_slab_timing_mark(pft_slab* s, int stage, int end)
{
  if (stage < 1 || stage > 5) return -2;
  if (!end && s->thead[stage] - s->ttail[stage] >= PFT_TRING) {
    int rc = timing_collect(s, true);   // ring full: read the oldest pairs before re-recording them
    if (rc) return rc;
  }
  hipEvent_t* ev = s->tev[stage][s->thead[stage] % PFT_TRING];
  if (!ev[0]) {
    HIPCHK(hipEventCreate(&ev[0]));
    HIPCHK(hipEventCreate(&ev[1]));
  }
  HIPCHK(hipEventRecord(ev[end ? 1 : 0], s->stream));
  if (end) s->thead[stage]++;
  return 0;
}

int pft_slab_timing_collect(pft_slab* s, double* ms, long* n)
{
  int rc = timing_collect(s, false);
  timing_hand_out(s, ms, n);
  return rc;
}

int pft_slab_timing_flush(pft_slab* s, double* ms, long* n)
{
  int rc = timing_collect(s, true);
  timing_hand_out(s, ms, n);
  return rc;
}

int pft_slab_can_speculate(const pft_slab* s) { return slab_kind(s) == KFUSED; }

// ---- gated steps (f4) ------------------------------------------------------------------------
// the device's x^0.2 correction (pow02_fix) compiled for the host: CPU tests check it against a
// high-precision reference with candidates one ulp off either way (tests/test_pow02.py)
double pft_pow02_fix(double x, double c) { return pow02_fix(x, c); }

int pft_slab_gate_config(pft_slab* s, double final_time, double delta, double h_min, int delta_local, int handle_nan)
{
  s->gate_final = final_time;
  s->gate_delta = delta;
  s->gate_hmin = h_min;
  s->gate_local = delta_local ? 1 : 0;
  s->gate_nan = handle_nan ? 1 : 0;
  return 0;
}

unsigned long long pft_slab_gate_arm(pft_slab* s, double t, double h)
{
  s->gate_arm_seq = ++s->gate_seq;
  s->gate_arm_t = t;
  s->gate_arm_h = h;
  return s->gate_arm_seq;
}

int pft_slab_gate_decision(pft_slab* s, unsigned long long seq, int* go, double* t, double* h)
{
  // the device's decision (gate_decide), published right after the error norm the host has read
  volatile unsigned long long* w = s->gate_pin + 4 * (seq % PFT_GATE_SLOTS);
  long spins = 0;
  unsigned long long v;
  while (((v = __atomic_load_n(&w[0], __ATOMIC_ACQUIRE)) & ~PFT_GATE_SKIP) != seq) {
    if (++spins < 200000) {
      __builtin_ia32_pause();
    } else if ((spins & 1023) == 0) {
      const hipError_t q = hipStreamQuery(s->stream);
      if (q != hipSuccess && q != hipErrorNotReady) return fail(q, "hipStreamQuery (gate decision poll)");
      if (q == hipSuccess && ((__atomic_load_n(&w[0], __ATOMIC_ACQUIRE) & ~PFT_GATE_SKIP) != seq))
        return fail(hipErrorUnknown, "gate decision never published");
      sched_yield();
    }
  }
  *go = v == seq;
  const unsigned long long tb = w[1], hb = w[2];
  memcpy(t, &tb, 8);
  memcpy(h, &hb, 8);
  return 0;
}

int pft_slab_gate_use(pft_slab* s, unsigned long long seq)
{
  s->gate_use_seq = seq;
  return 0;
}

int pft_slab_book_save(pft_slab* s, int which)
{
  if (which < 0 || which > 1) return -2;
  pft_slab::Book& b = s->book[which];
  b.pub_next = s->pub_next;
  b.pub_armed = s->pub_armed;
  b.pub_slot = s->pub_slot;
  b.eps_marked = s->eps_marked;
  b.defer_n = s->defer_n;
  b.defer_slot = s->defer_slot;
  return 0;
}

int pft_slab_book_load(pft_slab* s, int which)
{
  if (which < 0 || which > 1) return -2;
  const pft_slab::Book& b = s->book[which];
  // pub_next only moves forward: a discarded gated launch may still publish into its slot
  s->pub_next = std::max(s->pub_next, b.pub_next);
  s->pub_armed = b.pub_armed;
  s->pub_slot = b.pub_slot;
  s->eps_marked = b.eps_marked;
  s->defer_n = b.defer_n;
  s->defer_slot = b.defer_slot;
  return 0;
}

int pft_slab_stage_spec(pft_slab* s, double t_stage, int k_begin, int k_end)
{
  // stage 1 of the next step, K1' = f(t + h, x(t + h)), from XN into A1 (unused on the recompute
  // path) -- before the accept decision is known
  if (slab_kind(s) != KFUSED) return -2;
  return run_stage(s, 1, s->buf[PFT_BUF_XN], s->buf[PFT_BUF_A1], nullptr, t_stage, 0.0, 0.0, k_begin, k_end,
                   s->d.gl_static, KFUSED);
}

}  // extern "C"

// ---- pair kernels (merson_pair): stages 2+3 and 4+5 of a step, one launch each -------------

template <int SA, bool GLX, int LWP>
static void launch_pair_lwp(int mode, dim3 g, hipStream_t st, const PairArgs& a, const pft_consts& c)
{
  switch (mode) {
    case 0: merson_pair<SA, 0, GLX, LWP><<<g, PFT_PBLOCK, 0, st>>>(a, c); break;
    case 1: merson_pair<SA, 1, GLX, LWP><<<g, PFT_PBLOCK, 0, st>>>(a, c); break;
    case 2: merson_pair<SA, 2, GLX, LWP><<<g, PFT_PBLOCK, 0, st>>>(a, c); break;
    case 10: merson_pair<SA, 10, GLX, LWP><<<g, PFT_PBLOCK, 0, st>>>(a, c); break;
    case 11: merson_pair<SA, 11, GLX, LWP><<<g, PFT_PBLOCK, 0, st>>>(a, c); break;
  }
}

template <int SA, bool GLX>
static void launch_pair_mode(int mode, int lwp, dim3 g, hipStream_t st, const PairArgs& a, const pft_consts& c)
{
  if (lwp == 12) launch_pair_lwp<SA, GLX, 12>(mode, g, st, a, c);
  else launch_pair_lwp<SA, GLX, 22>(mode, g, st, a, c);
}

template <int SA, bool GLX>
static int pair_occupancy_mode(int mode)
{
  static int cache[12] = {0};
  int& n = cache[mode];
  if (n) return n;
  const void* f = mode == 0 ? (const void*)merson_pair<SA, 0, GLX, 22>
                : mode == 1 ? (const void*)merson_pair<SA, 1, GLX, 22>
                : mode == 2 ? (const void*)merson_pair<SA, 2, GLX, 22>
                : mode == 10 ? (const void*)merson_pair<SA, 10, GLX, 22>
                             : (const void*)merson_pair<SA, 11, GLX, 22>;
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, PFT_PBLOCK, 0) != hipSuccess || b < 1) b = 1;
  n = b;
  return n;
}

// the LDS row pitch (pairs) of a pair tile tx cells wide: 12 up to 20 cells, 22 up to 40
static int pair_lwp(int tx) { return tx <= 20 ? 12 : 22; }

// pair tile: tx cells (even) x ty rows; its R2 positions ((tx/2 + 2) pairs x (ty + 4) rows) one
// per thread, and the two LDS plane rings (rows of pair_lwp(tx) slots) within their halves
static bool pair_geometry_ok(int tx, int ty)
{
  const int lwp = pair_lwp(tx);
  // positions: one per thread, and up to PFT_PAIR_NEX more in the last ring row (LDS DMA)
  return tx >= 2 && tx % 2 == 0 && ty >= 1 &&
         (tx / 2 + 2) * (ty + 4) <= (lwp == 22 ? PFT_PBLOCK + PFT_PAIR_NEX : PFT_PBLOCK) &&
         (tx / 2 + 2) * (ty + 3) <= PFT_PBLOCK && tx / 2 + 2 <= 22 &&
         2 * PFT_PAIR_PADP + lwp * (ty + 4) <= PFT_PAIR_H && 2 * PFT_PAIR_PADP + lwp * (ty + 2) <= PFT_PAIR_HB &&
         (tx / 2) * ty <= PFT_PAIR_OPN;
}

// automatic tile: the fewest workgroups per plane (a workgroup-plane costs about the same whatever
// the tile's edge tiles hold), of those the one with the fewest idle tile cells, then the wider.
// n1 = 200 / 400: 40 x 20 cells (5 x 10 / 10 x 20 tiles, 484 of 512 threads evaluate stage A and
// 400 stage B, 16 positions of the last ring row DMA-staged; 40 x 19 before round 6); n1 = 100: 20 x 34 cells (5 x 3 tiles, 98% of their cells in the plane, against 18
// 34 x 19 tiles with the 22-pair pitch alone).  Returns the tiles per plane, 0 when no tile fits
// (n1 odd).
static long pair_geometry(int n1, int n2, int* tx_out, int* ty_out)
{
  long best = 0, best_idle = 0;
  int bx = 0, by = 0, bleg = 0;
  if (n1 < 2 || n1 % 2 || n2 < 1) return 0;
  for (int tx = 2; tx <= n1 + 1 && tx <= 40; tx += 2) {
    for (int ty = std::min(n2, PFT_PBLOCK); ty >= 1; --ty) {
      if (!pair_geometry_ok(tx, ty)) continue;
      const long nt = (long)((n1 + tx - 1) / tx) * ((n2 + ty - 1) / ty);
      const long idle = nt * tx * ty - (long)n1 * n2;
      // on a tie, a tile the round-5 limits allowed (one position per thread, 512 / 468 / 384 LDS
      // slots) keeps its place: the measured choices there (n1 = 100: 20 x 34) stay as they were
      const int leg = (tx / 2 + 2) * (ty + 4) <= PFT_PBLOCK && 2 * PFT_PAIR_PADP + pair_lwp(tx) * (ty + 4) <= 512 &&
                      2 * PFT_PAIR_PADP + pair_lwp(tx) * (ty + 2) <= 468 && (tx / 2) * ty <= 384;
      if (best == 0 || nt < best || (nt == best && (idle < best_idle || (idle == best_idle && leg >= bleg)))) {
        best = nt;
        best_idle = idle;
        bx = tx;
        by = ty;
        bleg = leg;
      }
    }
  }
  *tx_out = bx;
  *ty_out = by;
  return best;
}

// gl's terms of a pair launch (its K's are the literal zeros of dgl, equation.c:731,874), each the
// reference's expression with those zeros (hybrid2.c:388/428, 408/449, 521, 667), so every gl
// value the kernel forms is the reference's bit for bit
static void pair_gl_consts(PairArgs& a, int first, double em2)
{
  volatile double z = 0.0;    // evaluated at run time, operation by operation, like the kernels
  const double k = z;
  if (first == 2) {
    a.glA = k * a.cinA;                                   // stage 2: K1 h/3 + x
    a.glB = (k + k) * a.cinB;                             // stage 3: (K1 + K2) h/6 + x
  } else {
    a.glA = (k + 3.0 * k) * a.cinA;                       // stage 4: (K1 + 3 K3) h/8 + x
    a.glB = (0.5 * k - 1.5 * k + 2.0 * k) * a.cinB;       // stage 5: (0.5 K1 - 1.5 K3 + 2 K4) h + x
  }
  a.glX = a.coef * (0.5 * (k + k) + 2.0 * k);             // x(t+h) = x + h/3 (0.5 (K1 + K5) + 2 K4)
  a.evgl = em2 * fabs(0.2 * k - 0.9 * k + 0.8 * k - 0.1 * k);   // the error-norm term
}

static int run_pair(pft_slab* s, int first, double t_a, double t_b, double h, double coef, int k_begin,
                    int k_end)
{
  const int mode = s->d.calc_mode;
  if (mode != 0 && mode != 1 && mode != 2 && mode != 10 && mode != 11) return -2;
  if (first != 2 && first != 4) return -2;
  PairArgs a;
  memset(&a, 0, sizeof(a));
  // the buffers' pointers minus one plane: the far ghost plane below the first field (pair_load)
  a.x = s->buf[PFT_BUF_X] - s->plane;
  a.k1 = s->buf[PFT_BUF_K1] - s->plane;
  a.k3 = s->buf[PFT_BUF_K3] - s->plane;
  a.out = (first == 2 ? s->buf[PFT_BUF_K3] : s->buf[PFT_BUF_XN]) - s->plane;
  a.noise = s->noise;
  a.eps_bits = s->scratch;
  a.nonfinite = (unsigned int*)(s->scratch + 1);
  a.fs = s->fs;
  a.n1 = s->d.n1;
  a.n2 = s->d.n2;
  a.n3 = s->d.n3;
  a.plane = s->plane;
  a.has_below = s->d.has_below;
  a.has_above = s->d.has_above;
  // k_begin == PFT_K_BOUNDARY2: planes 0, 1 and n3-2, n3-1 in one launch (two 2-plane chunks);
  // PFT_K_INLINE: those chunks first, then the interior [2, n3 - 2), in one launch (bnd_mode 4)
  const bool bnd = k_begin == PFT_K_BOUNDARY2;
  bool ends = k_begin == PFT_K_ENDS_FIRST;
  const bool inl = k_begin == PFT_K_INLINE || ends;
  if (ends) {
    // the first and the last chunk must hold the two planes at each end (kz >= 2, a last chunk of
    // two planes or more) and leave a chunk between them; otherwise the two-plane boundary chunks
    const int n3 = s->d.n3;
    const int occ = first == 2 ? pair_occupancy_mode<2, false>(mode) : pair_occupancy_mode<4, false>(mode);
    const int kz = s->kz > 0 ? s->kz : chunk_kz(s, 14 + (first == 4 ? 1 : 0), occ, s->pair_ntile, n3, 3);
    const int nch = (n3 + kz - 1) / kz;
    if (kz < 2 || nch < 3 || n3 - (nch - 1) * kz < 2) ends = false;
  }
  if (inl && (!s->bdone || s->d.n3 < 5)) return -2;
  a.shards = s->eps_shards + (bnd ? PFT_EPS_SHARDS : 0);
  if (inl) {
    k_begin = ends ? 0 : 2;
    k_end = ends ? s->d.n3 : s->d.n3 - 2;
  }
  if (bnd || k_begin < 0) k_begin = 0;
  if (bnd || k_end < 0 || k_end > s->d.n3) k_end = s->d.n3;
  if (k_end <= k_begin) return 0;
  a.k_begin = k_begin;
  a.k_end = k_end;
  a.tx = s->pair_tx;
  a.ty = s->pair_ty;
  if (s->pair_ntile <= 0 || !pair_geometry_ok(a.tx, a.ty)) return -2;
  a.ntx = (a.n1 + a.tx - 1) / a.tx;
  a.ntile = a.ntx * ((a.n2 + a.ty - 1) / a.ty);
  const int nplanes = k_end - k_begin;
  if (s->kz > 0) {
    a.kz = s->kz;
  } else {
    // z-chunks as run_stage's cost model: a chunk of kz planes evaluates stage A on kz + 2 and
    // loads kz + 3; `occ` workgroups per CU (one: 141 KiB of LDS)
    const int occ = first == 2 ? pair_occupancy_mode<2, false>(mode) : pair_occupancy_mode<4, false>(mode);
    // end chunks first: at least three chunks, so that the first and last of a column are done
    // while the others still run (the exchange's copies go beside them)
    a.kz = chunk_kz(s, (ends ? 14 : 12) + (first == 4 ? 1 : 0), occ, a.ntile, nplanes, ends ? 3 : 1);
  }
  a.nchunk = (nplanes + a.kz - 1) / a.kz;
  a.kspan = a.kz;
  a.nint = a.ntile * a.nchunk;
  if (bnd) {
    a.kz = std::max(1, s->d.n3 - 2);
    a.kspan = 2;
    a.nchunk = s->d.n3 > 2 ? 2 : 1;
    a.nint = a.ntile * a.nchunk;
  }
  if (inl) {
    a.bdone = s->bdone;
    if (ends) {
      const int nb = std::min(a.nchunk, 2);
      a.nbw = nb * a.ntile;
      a.bends = 1;
      a.c0 = 1;
      a.nint = (a.nchunk - nb) * a.ntile;
    } else {
      a.nbw = 2 * a.ntile;
    }
  }
  const long nwg = (long)a.nbw + (long)a.nint;   // the launch's workgroups
  a.T_topA = t_a < s->c.phase_switch_time ? s->c.top_temp1 : s->c.top_temp2;
  a.T_topB = t_b < s->c.phase_switch_time ? s->c.top_temp1 : s->c.top_temp2;
  // exactly the solver's h/3.0, h/6.0 and h/8.0 (and run_stage's stage-input coefficients)
  a.cinA = first == 2 ? h / 3.0 : h / 8.0;
  a.cinB = first == 2 ? h / 6.0 : h;
  a.coef = coef;
  a.em0 = s->d.eps_mult[0];
  a.em1 = s->d.eps_mult[1];
  pair_gl_consts(a, first, s->d.eps_mult[2]);
  // gl's inputs are x itself (GLX): gl_static, or gl_keep with finite coefficients, where
  // glA + x == glB + x == x + glX == x for every gl value of x (no -0.0, no NaN: gl_clean)
  const bool glx = s->d.gl_static ||
                   (s->gl_keep && std::isfinite(a.cinA) && std::isfinite(a.cinB) && std::isfinite(coef));
  a.gl_keep = glx ? 1 : 0;
  s->pub_armed = 0;
  const int split_pub = s->split_pub;
  s->split_pub = 0;
  if (first == 4 && s->inkernel_pub && !bnd && ((k_begin == 0 && k_end == s->d.n3) || inl)) {
    const int j = (int)(s->pub_next % PFT_PUB_SLOTS);
    __atomic_store_n(&s->pub_ring[2 * j], PFT_PUB_SENTINEL, __ATOMIC_RELEASE);
    __atomic_store_n(&s->pub_ring[2 * j + 1], PFT_PUB_SENTINEL, __ATOMIC_RELEASE);
    const int rc = defer_arm(s, nwg, j, &a.part);
    if (rc) return rc;
    s->pub_armed = 1;
    s->pub_slot = j;
  } else if (first == 4 && s->inkernel_pub && bnd) {
    // split stage 4+5 (boundary, then interior: rk_solver do_pair): the boundary launch's partials
    // first, the interior's after them (the capacity for both now: no reallocation between the two
    // launches), reduced and published by the next stage-1 launch as for one launch
    const int j = (int)(s->pub_next % PFT_PUB_SLOTS);
    __atomic_store_n(&s->pub_ring[2 * j], PFT_PUB_SENTINEL, __ATOMIC_RELEASE);
    __atomic_store_n(&s->pub_ring[2 * j + 1], PFT_PUB_SENTINEL, __ATOMIC_RELEASE);
    const int rc = defer_arm(s, (long)a.ntile * a.nchunk, j, &a.part, (long)a.ntile * (a.nchunk + s->d.n3));
    if (rc) return rc;
    s->split_pub = 1;
  } else if (first == 4 && split_pub && !bnd && s->defer_n > 0 &&
             s->defer_n + (long)a.ntile * a.nchunk <= s->part_cap) {
    a.part = s->part + 2 * (long)s->defer_n;
    s->defer_n += a.ntile * a.nchunk;
    s->pub_armed = 1;
    s->pub_slot = s->defer_slot;
  }
  const dim3 g((unsigned)nwg);
  hipStream_t st = s->stream;
  // bnd_mode 1, 2: the boundary launch beside the interior one.  On a 400 x 400 plane the interior
  // holds one workgroup per tile column, 220 of 256 CUs: the boundary's workgroups take the CUs it
  // leaves and the copies start while the interior still runs.  An interior launch of more
  // workgroups than CUs (several rounds, the 318^2 and 252^2 planes) leaves CUs only in its last
  // round, and beside is still no slower there than before (profiles/r05_ce_shapes.txt)
  const bool beside = bnd && s->bnd_mode != 0;
  if (beside) {
    HIPCHK(hipEventRecord(s->ev_pre, s->stream));
    HIPCHK(hipStreamWaitEvent(s->bnd, s->ev_pre, 0));
    st = s->bnd;
  }
  const int lwp = pair_lwp(a.tx);
  if (first == 2) {
    if (glx) launch_pair_mode<2, true>(mode, lwp, g, st, a, s->c);
    else launch_pair_mode<2, false>(mode, lwp, g, st, a, s->c);
  } else {
    if (glx) launch_pair_mode<4, true>(mode, lwp, g, st, a, s->c);
    else launch_pair_mode<4, false>(mode, lwp, g, st, a, s->c);
  }
  HIPCHK(hipGetLastError());
  if (beside) {
    HIPCHK(hipEventRecord(s->ev_bnd, s->bnd));
    s->bnd_pending = 1;
  }
  if (inl) {
    s->bdone_target += (unsigned long long)a.nbw;
    s->inline_pending = 1;
    // the copies' trigger, on the comm stream at once: queued now, it is normally dispatched while
    // the previous launch still runs and sits on its CU before this launch fills the chip (pair 4+5
    // at 256 VGPRs leaves no room beside its workgroups: a trigger queued later waited for a CU
    // until this launch drained -- the copies then ran after it)
    if (s->trig_early) {
      bnd_trigger_kernel<<<1, 64, 0, s->comm>>>(s->bdone, s->bdone_target);
      HIPCHK(hipGetLastError());
    }
  }
  return 0;
}

extern "C" {

int pft_slab_set_pair(pft_slab* s, int on)
{
  if (on < 0 || on > 2) return -2;
  if (!s->pair_env) s->pair_on = on;
  return 0;
}

int pft_slab_pair_ok(const pft_slab* s)
{
  // automatic: slabs of at least PFT_PAIR_MIN_CELLS_PER_CU cells per CU.  Measured (A/B, one box):
  // 400^3 +28% (round 3), 200^3 (2 M cells, 7.8 Ki per CU) +6% since the 12-pair row pitch of
  // 100-wide planes (round 4: 14 384 against 13 575 Mcells*steps/s), 100^3 -28% (one workgroup
  // per CU marching 3-5 planes, two of them stage-A-only, against one plane per workgroup)
  if (s->pair_on == 1 && (double)s->plane * s->d.n3 < (double)s->n_cu * PFT_PAIR_MIN_CELLS_PER_CU) return 0;
  // z-neighbours: the two-plane halo (pft_comm_halo_deep) needs n3 >= 2, and stage A on a ghost
  // plane would need the neighbour's u_noise there (not exchanged: one launch per stage then)
  const bool nb = s->d.has_below || s->d.has_above;
  if (nb && (s->d.n3 < 2 || s->noise)) return 0;
  // (merson_pair addresses a field with 32-bit byte offsets, and the extra positions' LDS DMA the
  // three fields of a buffer from one base: 3 fields < 4 GiB, 178 M cells per slab)
  return s->pair_on && slab_kind(s) == KFUSED &&
         3.0 * (double)s->fs * 8.0 < 4294967296.0 && s->pair_ntile > 0;
}

int pft_slab_pair_geometry(const pft_slab* s, int* tx, int* ty)
{
  *tx = s->pair_tx;
  *ty = s->pair_ty;
  return s->pair_ntile > 0 ? 0 : -2;
}

int pft_slab_pair(pft_slab* s, int first, double t_a, double t_b, double h, double coef)
{
  return pft_slab_pair_range(s, first, t_a, t_b, h, coef, -1, -1);
}

int pft_slab_boundary_inline(const pft_slab* s)
{
  return s->bnd_mode >= 4 && s->bdone && s->d.n3 >= 5 && slab_kind(s) == KFUSED
             ? (s->bnd_mode == 5 ? PFT_K_ENDS_FIRST : PFT_K_INLINE)
             : 0;
}

int pft_slab_stage_inline(const pft_slab* s) { return s->stage_inline ? pft_slab_boundary_inline(s) : 0; }

int pft_slab_pair_inline(const pft_slab* s, int first)
{
  const int m = pft_slab_boundary_inline(s);
  if (!m) return 0;
  // A/B: PFT_CE_BND23 / PFT_CE_BND45 = 4 or 5 overrides the placement of one pair kernel
  const char* e = getenv(first == 2 ? "PFT_CE_BND23" : "PFT_CE_BND45");
  if (e && atoi(e) == 4) return PFT_K_INLINE;
  if (e && atoi(e) == 5) return PFT_K_ENDS_FIRST;
  // placement 5: end chunks first where the one-wave trigger kernel fits on a CU beside the pair
  // kernel's workgroup (pair 2+3: 216-221 VGPRs, 126 KiB of LDS).  Pair 4+5 at 256 VGPRs (every
  // calc mode but 2, scripts/kernel_resources.py) fills each SIMD's register file, so the trigger
  // holds a CU of its own for as long as it waits -- half the launch with end chunks, and one CU
  // fewer in one XCD costs that XCD a round of workgroups (400 x 400 x 100: 125 per XCD, 4 rounds
  // on 32 CUs, 5 on 31; pair 4+5 0.479 against 0.404 ms, profiles/r06_ce_inline.txt).  There the
  // two-plane boundary chunks (placement 4) free CUs within a few plane steps and the trigger ends
  // with them.
  if (m == PFT_K_ENDS_FIRST && first == 4 && s->d.calc_mode != 2) return PFT_K_INLINE;
  return m;
}

int pft_slab_pair_range(pft_slab* s, int first, double t_a, double t_b, double h, double coef, int k_begin,
                        int k_end)
{
  if (!pft_slab_pair_ok(s)) return -2;
  return run_pair(s, first, t_a, t_b, h, coef, k_begin, k_end);
}

int pft_slab_swap_buffers(pft_slab* s, int a, int b)
{
  if (a < 0 || a >= PFT_BUF_COUNT || b < 0 || b >= PFT_BUF_COUNT) return -2;
  double* t = s->buf[a];
  s->buf[a] = s->buf[b];
  s->buf[b] = t;
  const int p = s->phys[a];
  s->phys[a] = s->phys[b];
  s->phys[b] = p;
  return 0;
}

int pft_slab_accept(pft_slab* s) { return pft_slab_swap_buffers(s, PFT_BUF_X, PFT_BUF_XN); }

static int ensure_rbuf(pft_slab* s)
{
  // two slots (exchange sequence number parity): a neighbour can be one exchange ahead -- its
  // next put needs only our flag of this exchange, which we raise before copying its planes out
  if (!s->rbuf) HIPCHK(hipExtMallocWithFlags((void**)&s->rbuf, sizeof(double) * 24 * (size_t)s->plane, hipDeviceMallocUncached));
  return 0;
}

int pft_slab_ipc_export(pft_slab* s, void* handles)
{
  hipIpcMemHandle_t* h = (hipIpcMemHandle_t*)handles;
  int rc = ensure_rbuf(s);
  if (rc) return rc;
  for (int b = 0; b < PFT_BUF_COUNT; ++b) HIPCHK(hipIpcGetMemHandle(&h[b], s->buf0[b]));
  HIPCHK(hipIpcGetMemHandle(&h[PFT_BUF_COUNT], s->sig));
  HIPCHK(hipIpcGetMemHandle(&h[PFT_BUF_COUNT + 1], s->rbuf));
  return 0;
}

int pft_ipc_staged_env(void)
{
  const char* e = getenv("PFT_IPC_STAGED");
  return e && atoi(e) == 1;
}

int pft_slab_ipc_set_peer(pft_slab* s, int side, const void* handles, int n3, long fs, int remote,
                          int peer_staged)
{
  if (side < 0 || side > 1) return -2;
  SlabPeer& p = s->peer[side];
  if (p.on) return -2;                  // pft_slab_ipc_close first
  if (!handles) {
    // self exchange (diagnostic, one slab): the planes land in the slab's own ghost planes, which a
    // single slab never reads (mirror bottom, Dirichlet top)
    int rc = ensure_rbuf(s);
    if (rc) return rc;
    for (int b = 0; b < PFT_BUF_COUNT; ++b) p.base[b] = s->buf0[b] + s->plane;
    p.sig = s->sig;
    p.rbuf = s->rbuf;
    p.staged = pft_ipc_staged_env();
    p.n3 = s->d.n3;
    p.fs = s->fs;
    p.opened = 0;
    p.on = 1;
    return 0;
  }
  const hipIpcMemHandle_t* h = (const hipIpcMemHandle_t*)handles;
  for (int b = 0; b <= PFT_BUF_COUNT + 1; ++b) {
    void* ptr = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&ptr, h[b], hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      for (int q = 0; q < b && q < PFT_BUF_COUNT; ++q) (void)hipIpcCloseMemHandle(p.base[q] - s->plane);
      if (b > PFT_BUF_COUNT) (void)hipIpcCloseMemHandle(p.sig);
      return fail(e, "hipIpcOpenMemHandle");
    }
    if (b < PFT_BUF_COUNT) p.base[b] = (double*)ptr + s->plane;   // the neighbour's buffer pointer
    else if (b == PFT_BUF_COUNT) p.sig = (unsigned long long*)ptr;
    else p.rbuf = (double*)ptr;
  }
  p.n3 = n3;
  p.fs = fs;
  p.remote = remote ? 1 : 0;   // the caller compared the GPUs' identities (pft_hip_device_ident)
  // A neighbour on another GPU writes into our receive buffer (uncached) rather than our ghost
  // planes, and we copy it in after the flag wait: no L2 of ours can hold a stale line of what it
  // wrote.  Both sides take the same decision: remote is symmetric, and the
  // env (the test hook that stages between processes on one GPU) counts if either side set it --
  // a sender putting into ghost planes that the receiver overwrites from its receive buffer, or
  // the other way round, would corrupt the halo without any error.
  p.staged = p.remote || pft_ipc_staged_env() || peer_staged;
  p.opened = 1;
  p.on = 1;
  return 0;
}

int pft_slab_ipc_close(pft_slab* s)
{
  if (s->ipc_poisoned == 1) {
    // the flags were forced past every sequence number: back to 0 for the next attach (the compute
    // stream has drained, slab_wait)
    (void)hipStreamSynchronize(s->stream);
    (void)hipStreamSynchronize(s->side);
    if (s->bnd) (void)hipStreamSynchronize(s->bnd);

    (void)hipStreamSynchronize(s->comm);
    HIPCHK(hipMemset(s->sig, 0, 2 * sizeof(unsigned long long)));
    HIPCHK(hipDeviceSynchronize());
    s->ipc_poisoned = 0;
  }
  if ((s->peer[0].on && s->peer[0].opened) || (s->peer[1].on && s->peer[1].opened)) {
    // the copy-engine exchange's streams write into the mappings about to be closed: drained first
    // (they wait only on compute-stream work, which the detach's pft_slab_sync has drained)
    if (s->comm) (void)hipStreamSynchronize(s->comm);
    if (s->side) (void)hipStreamSynchronize(s->side);
  }
  for (int side = 0; side < 2; ++side) {
    SlabPeer& p = s->peer[side];
    if (p.on && p.opened) {
      for (int b = 0; b < PFT_BUF_COUNT; ++b) (void)hipIpcCloseMemHandle(p.base[b] - s->plane);
      (void)hipIpcCloseMemHandle(p.sig);
      (void)hipIpcCloseMemHandle(p.rbuf);
    }
    memset(&p, 0, sizeof(p));
  }
  return 0;
}

int pft_slab_halo_put(pft_slab* s, int role, int f0, int f1, unsigned long long seq)
{
  return pft_slab_halo_put2(s, role, f0, f1, 0, seq);
}

double* pft_slab_far(pft_slab* s, int which, int q, int side)
{
  if (which < 0 || which >= PFT_BUF_COUNT || q < 0 || q > 2 || side < 0 || side > 1) return nullptr;
  return s->buf[which] + q * s->fs + (side ? (long)(s->d.n3 + 2) * s->plane : -(long)s->plane);
}

int pft_slab_halo_put2(pft_slab* s, int role, int f0, int f1, int deep, unsigned long long seq)
{
  if (role < 0 || role >= PFT_BUF_COUNT || f0 < 0 || f1 > 3 || f1 <= f0) return -2;
  if (s->ipc_poisoned) return slab_poisoned(s, "pft_slab_halo_put2");
  s->put_role = role;
  s->put_f0 = f0;
  s->put_f1 = f1;
  s->put_deep = deep ? 1 : 0;
  if (s->drop_puts) return 0;
  const int ph = s->phys[role];
  PutArgs a;
  memset(&a, 0, sizeof(a));
  a.src = s->buf[role];
  a.fs = s->fs;
  a.plane = s->plane;
  a.n3 = s->d.n3;
  a.f0 = f0;
  a.nf = f1 - f0;
  // staged: into the neighbour's receive buffer [side][depth][field][plane] -- the neighbour below
  // receives our planes as "from above" (side 1), the one above as "from below" (side 0)
  const long P = s->plane;
  const long slot = (long)(seq & 1) * 12 * P;   // the receive-buffer slot of this exchange
  if (s->peer[0].on) {
    a.dlo = s->peer[0].staged ? s->peer[0].rbuf + slot + (1 * 2 + 0) * 3 * P : s->peer[0].base[ph] + (long)(s->peer[0].n3 + 1) * P;
    a.dlo_fs = s->peer[0].staged ? P : s->peer[0].fs;
  }
  if (s->peer[1].on) {
    a.dhi = s->peer[1].staged ? s->peer[1].rbuf + slot + (0 * 2 + 0) * 3 * P : s->peer[1].base[ph];
    a.dhi_fs = s->peer[1].staged ? P : s->peer[1].fs;
  }
  if (!a.dlo && !a.dhi) return 0;
  if (deep) {
    // the second boundary planes into the neighbours' far ghost planes (pft_slab_far layout)
    a.deep = 1;
    if (s->peer[0].on)
      a.flo = s->peer[0].staged ? s->peer[0].rbuf + slot + (1 * 2 + 1) * 3 * P : s->peer[0].base[ph] + (long)(s->peer[0].n3 + 2) * P;
    if (s->peer[1].on) a.fhi = s->peer[1].staged ? s->peer[1].rbuf + slot + (0 * 2 + 1) * 3 * P : s->peer[1].base[ph] - P;
  }
  const long n = (deep ? 4L : 2L) * a.nf * s->plane;
  const int blocks = (int)std::min<long>(1024, std::max<long>(1, (n + 255) / 256));
  halo_put_kernel<<<blocks, 256, 0, s->stream>>>(a);
  HIPCHK(hipGetLastError());
  return pft_slab_halo_signal(s, seq);
}

#define PFT_SEQTAB 4096

// The ipc exchange on the copy engines (SDMA): after the launch that wrote the boundary planes (an
// event on the compute stream), the comm stream copies them into the neighbours' ghost (and far
// ghost) planes -- or their receive buffers when staged -- with hipMemcpyDeviceToDeviceNoCU, then
// raises the neighbours' flags with 8-byte copies of the sequence number from seqtab.  No kernel:
// the copies need no CU, so they run beside the interior launch that holds every CU's LDS (a blit
// kernel, or RCCL's, waits for that launch to end: profiles/r05_sdma_probe.txt).  The receiver
// side is unchanged (pft_slab_halo_wait: the compute stream waits for the flags; staged: the
// receive kernel), so a sender may use either put.
int pft_slab_halo_put_ce(pft_slab* s, int role, int f0, int f1, int deep, unsigned long long seq)
{
  if (role < 0 || role >= PFT_BUF_COUNT || f0 < 0 || f1 > 3 || f1 <= f0 || seq == 0) return -2;
  if (s->ipc_poisoned) return slab_poisoned(s, "pft_slab_halo_put_ce");
  const int marked = s->ce_marked;
  s->ce_marked = 0;
  s->put_role = role;
  s->put_f0 = f0;
  s->put_f1 = f1;
  s->put_deep = deep ? 1 : 0;
  if (s->drop_puts) return 0;
  if (!s->peer[0].on && !s->peer[1].on) return 0;
  if (!s->seqtab) {
    HIPCHK(hipMalloc((void**)&s->seqtab, sizeof(unsigned long long) * PFT_SEQTAB));
    HIPCHK(hipHostMalloc((void**)&s->seqhost, 2 * sizeof(unsigned long long) * PFT_SEQTAB, hipHostMallocDefault));
    for (int i = 0; i < 2; ++i) HIPCHK(hipEventCreateWithFlags(&s->ev_seq[i], hipEventDisableTiming));
    s->seq_base = ~0ULL;
    // test hook PFT_CE_SEQTAB=n (2..4096): a table of n numbers, refilled every n exchanges
    const char* et = getenv("PFT_CE_SEQTAB");
    s->seq_n = (et && atoi(et) >= 2 && atoi(et) <= PFT_SEQTAB) ? atoi(et) : PFT_SEQTAB;
    // the flags behind an explicit completion of the plane copies (default 1; PFT_CE_FENCE=0: each
    // flag copy right behind its planes on the same stream, relying on the in-order SDMA queue)
    const char* ef = getenv("PFT_CE_FENCE");
    s->ce_fence = !(ef && atoi(ef) == 0);
    for (int i = 0; i < 2; ++i) HIPCHK(hipEventCreateWithFlags(&s->ev_planes[i], hipEventDisableTiming));
  }
  const int NSEQ = s->seq_n;
  if (s->seq_base == ~0ULL || seq <= s->seq_base || seq > s->seq_base + NSEQ) {
    // the next block of sequence numbers, from the pinned half not used by the previous refill
    s->seq_base = (seq - 1) / NSEQ * NSEQ;
    s->seq_half ^= 1;
    if (s->ce_streams != 1) {
      // the side stream's last flag copy reads the old table: the refill (comm stream) waits for it
      HIPCHK(hipEventRecord(s->ev_side, s->side));
      HIPCHK(hipStreamWaitEvent(s->comm, s->ev_side, 0));
    }
    // this pinned half was last read by the refill copy two refills ago: the host rewrites it only
    // once that copy has run (with a small table -- the PFT_CE_SEQTAB test hook -- the speculative
    // pipeline can hold that many exchanges queued)
    // (bounded like every host wait with ipc peers: a lost peer can hold that copy's stream)
    {
      const int wrc = slab_wait(s, s->ev_seq[s->seq_half], "pft_slab_halo_put_ce (seqtab refill)");
      if (wrc) return wrc;
    }
    unsigned long long* h = s->seqhost + (size_t)s->seq_half * PFT_SEQTAB;
    for (int i = 0; i < NSEQ; ++i) h[i] = s->seq_base + 1 + i;
    HIPCHK(hipMemcpyAsync(s->seqtab, h, sizeof(unsigned long long) * NSEQ, hipMemcpyHostToDevice, s->comm));
    HIPCHK(hipEventRecord(s->ev_seq[s->seq_half], s->comm));
    if (s->ce_streams != 1) {
      // the side stream's flag copies read the new table: this exchange's (and so every later one's)
      // follow the refill.  (An event on every exchange instead held each side flag behind the comm
      // stream's copies and put a marker between the comm stream's last copy and its flag: ~10-20
      // us later flags, profiles/r05_ce_trace_pipe.txt.)
      HIPCHK(hipEventRecord(s->ev_copy, s->comm));
      HIPCHK(hipStreamWaitEvent(s->side, s->ev_copy, 0));
    }
  }
  // the planes to the neighbour below go on the comm stream, to the one above on the side stream
  // (two copy engines; ce_streams = 1: all on the comm stream), each followed by its neighbour's
  // flag.  (Four streams, a side's copies alternating between two, measured slower: 11 300-12 600
  // against 16 000 Mcells*steps/s on the 800^3 rank slab, profiles/r05_ce_ab.txt; removed.)
  hipStream_t cs[2] = {s->comm, s->ce_streams == 1 ? s->comm : s->side};
  if (s->inline_pending) {
    // inline boundary: the copies start once the launch's boundary workgroups have counted
    // themselves -- not at its end, and with no event on the compute stream between them
    // (trig_early: the trigger is on the comm stream already, queued with the launch)
    s->inline_pending = 0;
    if (!s->trig_early) {
      bnd_trigger_kernel<<<1, 64, 0, cs[0]>>>(s->bdone, s->bdone_target);
      HIPCHK(hipGetLastError());
    }
    if (cs[1] != cs[0]) {
      HIPCHK(hipEventRecord(s->ev_trig, cs[0]));
      HIPCHK(hipStreamWaitEvent(cs[1], s->ev_trig, 0));
    }
  } else {
    hipEvent_t ready = s->bnd_pending ? s->ev_bnd : s->ev_order[0];
    if (!s->bnd_pending && !marked) HIPCHK(hipEventRecord(s->ev_order[0], s->stream));
    HIPCHK(hipStreamWaitEvent(cs[0], ready, 0));
    if (cs[1] != cs[0]) HIPCHK(hipStreamWaitEvent(cs[1], ready, 0));
  }
  const int ph = s->phys[role];
  const long P = s->plane, n3 = s->d.n3;
  const long slot = (long)(seq & 1) * 12 * P;
  const size_t pb = sizeof(double) * (size_t)P;
  for (int side = 0; side < 2; ++side) {
    const SlabPeer& p = s->peer[side];
    if (!p.on) continue;
    for (int q = f0; q < f1; ++q) {
      const double* src = s->buf[role] + q * s->fs;
      if (!p.staged) {
        // below: our planes 1 (, 2) into its ghost n3'+1 (, far n3'+2); above: our planes (n3-1,) n3
        // into its (far -1,) ghost 0 -- contiguous on both ends
        double* dst = side == 0 ? p.base[ph] + q * p.fs + (p.n3 + 1) * P : p.base[ph] + q * p.fs - (deep ? P : 0);
        const double* sp = side == 0 ? src + P : src + (deep ? n3 - 1 : n3) * P;
        HIPCHK(hipMemcpyAsync(dst, sp, (deep ? 2 : 1) * pb, hipMemcpyDeviceToDeviceNoCU, cs[side]));
      } else {
        // its receive buffer [slot][side][depth][field][plane]: the neighbour below receives our
        // planes as "from above" (side 1), the one above as "from below" (side 0)
        for (int d = 0; d < (deep ? 2 : 1); ++d) {
          double* dst = p.rbuf + slot + ((long)((side == 0 ? 1 : 0) * 2 + d) * 3 + q) * P;
          const double* sp = side == 0 ? src + (1 + d) * P : src + (n3 - d) * P;
          HIPCHK(hipMemcpyAsync(dst, sp, pb, hipMemcpyDeviceToDeviceNoCU, cs[side]));
        }
      }
    }
  }
  const unsigned long long* sv = s->seqtab + (seq - 1 - s->seq_base);
  // The neighbour reads the planes once it sees the flag, so the flag must not land before them.
  // ce_fence (default): the flag copy goes on a stream of its own behind an event recorded after
  // the side's plane copies.  The runtime turns that event wait into a dependency on the copies'
  // completion signal (hsa_amd_memory_async_copy, hsa_ext_amd.h: "the copy will start after every
  // [dependent] signal has been observed with the value 0", and the completion signal is
  // decremented "when the copy operation is finished"), so the flag copy starts only after the
  // plane copies have finished -- an ordering the HSA interface states, where a flag copy right
  // behind them on the same stream relies on the SDMA queue retiring its writes in order (not a
  // documented property across xGMI; PFT_CE_FENCE=0 restores that form for A/B).  The receiver's
  // side is the system-scope acquire load of the flag in halo_wait_kernel (hsa_ext_amd.h asks the
  // receiving device for a system-scope acquire before it uses a copy's destination).
  // No stream is added for it: a process has 4 hardware queues (GPU_MAX_HW_QUEUES) and already 4
  // streams (compute, boundary, comm, side); a fifth and sixth share queues with them, and their
  // waits then hold up unrelated work -- one flag stream per side measured that way (DESIGN
  // section 6).  So each side's flag goes on the OTHER copy stream, behind an event after this
  // side's planes: with two neighbours both flags land after both sides' planes (the two run side
  // by side, of equal size), each ordered after its own planes by the event.  With one copy stream
  // (ce_streams 1) the stream order is all there is.
  hipStream_t fs[2] = {cs[0], cs[1]};
  if (s->ce_fence && cs[1] != cs[0]) {
    for (int side = 0; side < 2; ++side)
      if (s->peer[side].on) HIPCHK(hipEventRecord(s->ev_planes[side], cs[side]));
    for (int side = 0; side < 2; ++side)
      if (s->peer[side].on) {
        fs[side] = cs[1 - side];
        HIPCHK(hipStreamWaitEvent(fs[side], s->ev_planes[side], 0));
      }
  }
  if (s->peer[0].on) HIPCHK(hipMemcpyAsync(s->peer[0].sig + 1, sv, 8, hipMemcpyDeviceToDeviceNoCU, fs[0]));
  if (s->peer[1].on) HIPCHK(hipMemcpyAsync(s->peer[1].sig + 0, sv, 8, hipMemcpyDeviceToDeviceNoCU, fs[1]));
  return 0;
}

int pft_slab_halo_mark(pft_slab* s)
{
  if (s->ipc_poisoned) return slab_poisoned(s, "pft_slab_halo_mark");
  if (!s->bnd_pending && !s->inline_pending) HIPCHK(hipEventRecord(s->ev_order[0], s->stream));
  s->ce_marked = 1;
  return 0;
}

int pft_slab_set_boundary_stream(pft_slab* s, int on)
{
  if (on && !s->bnd) {
    int lo = 0, hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCHK(hipStreamCreateWithPriority(&s->bnd, hipStreamNonBlocking, hi));
    HIPCHK(hipEventCreateWithFlags(&s->ev_bnd, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s->ev_pre, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s->ev_copy, hipEventDisableTiming));
  }
  if (on && !s->ev_copy) HIPCHK(hipEventCreateWithFlags(&s->ev_copy, hipEventDisableTiming));
  // bnd_mode 2: the pair kernels' boundary launch on its own stream beside their interior launch
  // (run_pair); a stage launch's boundary runs before its interior.  3 (round 5's default): the
  // boundary pipeline -- as 2, and the halo waits on the boundary stream (pft_slab_halo_wait), so
  // that no pair interior launch waits for a neighbour's flag (profiles/r05_ce_shapes.txt: +1% over 2
  // on one GPU).  5 (default since round 6): one pair launch per exchange, no boundary launch --
  // pair 2+3 with every tile column's first and last z-chunk leading the grid (PFT_K_ENDS_FIRST),
  // pair 4+5 with two-plane boundary chunks leading its interior chunks (PFT_K_INLINE, see
  // pft_slab_pair_inline); the copies start behind bnd_trigger_kernel once those workgroups are
  // done, while the rest of the launch runs.  The interior launch of 2 / 3 holds the CUs for
  // several rounds of workgroups on the driver's N > 1 slabs, so their boundary launch beside it
  // ran late and its copies after it (profiles/r06_ce_shapes.txt).  4: placement 4 for both pairs.
  // Stage launches keep their boundary first (inline with PFT_CE_STAGE_INLINE=1: slower, the
  // boundary workgroups' write-backs in a 3-workgroups-per-CU launch).  Env overrides for A/B
  // (profiles/r05_ce_ab.txt, r05_ce_shapes.txt, r06_ce_shapes.txt): PFT_CE_BND=2 the
  // waits on the compute stream, 0 every boundary before its interior, 1 every one beside (slower:
  // a stage launch's interior fills the chip, the two launches' workgroups are dealt interleaved
  // and the boundary ends late, profiles/r05_ce_trace_bnd.txt); PFT_CE_STREAMS=1 puts every copy
  // on the comm stream (slower)
  const char* eb = getenv("PFT_CE_BND");
  const char* es = getenv("PFT_CE_STREAMS");
  s->bnd_mode = !on ? 0 : eb && atoi(eb) >= 0 && atoi(eb) <= 5 ? atoi(eb) : 5;
  if (s->bnd_mode >= 4 && !s->bdone) {
    HIPCHK(hipMalloc((void**)&s->bdone, 64));
    HIPCHK(hipMemsetAsync(s->bdone, 0, 64, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    s->bdone_target = 0;
    HIPCHK(hipEventCreateWithFlags(&s->ev_trig, hipEventDisableTiming));
  }
  s->inline_pending = 0;
  {
    const char* et = getenv("PFT_CE_TRIG");
    const char* esi = getenv("PFT_CE_STAGE_INLINE");
    s->trig_early = et ? atoi(et) != 0 : 1;
    s->stage_inline = esi ? atoi(esi) != 0 : 0;
  }
  {
    // CUs reserved for the boundary launches (PFT_CE_RESERVE=R): the compute stream is re-created
    // with a CU mask that leaves R CUs out, so an interior launch of several rounds of workgroups
    // can never hold the CUs the boundary launch beside it needs.  R/8 per XCD, chosen so that
    // either numbering of the mask (CU-major per XCD or XCD-interleaved) spreads them evenly.
    const char* er = getenv("PFT_CE_RESERVE");
    const int want = on && s->bnd_mode >= 2 && er ? atoi(er) : 0;
    if (want != s->cu_reserved && want >= 0 && want <= 32 && want % 8 == 0 && s->n_cu == 256) {
      uint32_t mask[8];
      for (int w = 0; w < 8; ++w) mask[w] = ~0u;
      for (int x = 0; x < 8; ++x)
        for (int j = 0; j < want / 8; ++j) {
          const int bit = 32 * x + 8 * j + x;   // residue x mod 8, in the block of 32 numbered x
          mask[bit / 32] &= ~(1u << (bit % 32));
        }
      hipStream_t ns = nullptr;
      HIPCHK(hipStreamSynchronize(s->stream));
      HIPCHK(hipExtStreamCreateWithCUMask(&ns, 8, mask));
      HIPCHK(hipStreamDestroy(s->stream));
      s->stream = ns;
      s->cu_reserved = want;
    }
  }
  s->ce_streams = es && atoi(es) == 1 ? 1 : 2;
  if (s->ce_streams == 2 && !s->ev_copy) HIPCHK(hipEventCreateWithFlags(&s->ev_copy, hipEventDisableTiming));
  if (!s->ev_side) HIPCHK(hipEventCreateWithFlags(&s->ev_side, hipEventDisableTiming));
  if (!s->ev_join) HIPCHK(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming));
  s->bnd_pending = 0;
  return 0;
}

int pft_slab_halo_signal(pft_slab* s, unsigned long long seq)
{
  if (s->ipc_poisoned) return slab_poisoned(s, "pft_slab_halo_signal");
  if (s->drop_puts) return 0;
  unsigned long long* slo = s->peer[0].on ? s->peer[0].sig + 1 : nullptr;   // below: its "from above"
  unsigned long long* shi = s->peer[1].on ? s->peer[1].sig + 0 : nullptr;   // above: its "from below"
  if (!slo && !shi) return 0;
  halo_signal_kernel<<<1, 64, 0, s->stream>>>(slo, shi, seq,
                                              s->peer[0].remote || s->peer[1].remote || s->peer[0].staged || s->peer[1].staged);
  HIPCHK(hipGetLastError());
  return 0;
}

int pft_slab_halo_wait(pft_slab* s, unsigned long long seq)
{
  // flags [0] (from below) and [1] (from above): the stream goes on once both planes are in
  if (s->ipc_poisoned) return slab_poisoned(s, "pft_slab_halo_wait");
  // the boundary pipeline (bnd_mode 3): after a boundary launch beside the interior, the flags are
  // waited for on the boundary stream -- only the next boundary launch (after this wait on that
  // stream) reads ghost planes; the next interior launch waits for this boundary launch alone
  hipStream_t ws = s->stream;
  if (s->bnd_pending) {
    // the boundary launch ran beside the interior one: its planes are the next launch's input
    HIPCHK(hipStreamWaitEvent(s->stream, s->ev_bnd, 0));
    s->bnd_pending = 0;
    if (s->bnd_mode == 3) ws = s->bnd;
  } else if (s->bnd_split && s->bnd_mode == 3 && s->bnd) {
    // a boundary launch before its interior (stage 1): its flags too are waited for on the
    // boundary stream, which the next boundary launch follows (run_pair beside, run_stage joins)
    ws = s->bnd;
  }
  s->bnd_split = 0;
  int sides = 0;
  WaitArgs w;
  memset(&w, 0, sizeof(w));
  w.seq = seq;
  for (int side = 0; side < 2; ++side) {
    if (!s->peer[side].on) continue;
    (side == 0 ? w.f0 : w.f1) = s->sig + side;
    if (s->peer[side].staged) sides |= 1 << side;
  }
  if (!w.f0 && !w.f1) return 0;
  int local_staged = 0;
  for (int side = 0; side < 2; ++side)
    if (((sides >> side) & 1) && !s->peer[side].remote) local_staged = 1;
  int blocks = 1;
  if (sides) {
    // staged: what the neighbours put into the receive buffer, into the ghost planes of the
    // exchange's buffer (the one the last halo_put2 sent: every rank runs the same sequence)
    RecvArgs& r = w.r;
    r.rbuf = s->rbuf + (long)(seq & 1) * 12 * s->plane;
    r.dst = s->buf[s->put_role];
    r.fs = s->fs;
    r.plane = s->plane;
    r.n3 = s->d.n3;
    r.f0 = s->put_f0;
    r.nf = s->put_f1 - s->put_f0;
    r.depth = s->put_deep ? 2 : 1;
    r.sides = sides;
    w.recv = 1;
    blocks = pft_halo_wait_blocks(4L * r.nf * s->plane, local_staged, s->gpu_ranks, ws == s->bnd);
  }
  if (s->wait_streamops) {
    // A/B (PFT_WAIT_STREAMOPS=1): the runtime's stream waits, then a separate receive launch
    for (int side = 0; side < 2; ++side)
      if (s->peer[side].on) HIPCHK(hipStreamWaitValue64(ws, s->sig + side, seq, hipStreamWaitValueGte, ~0ULL));
    if (sides) halo_recv_kernel<<<blocks, 256, 0, ws>>>(w.r);
  } else {
    halo_wait_kernel<<<blocks, 256, 0, ws>>>(w);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// Workgroups of one halo_wait_kernel launch with a staged receive of n doubles.  Every block spins
// on the flags before it copies, so the count bounds the CUs a wait can hold while the neighbour
// whose launch raises the flag may need them:
//  - a staged neighbour on this same GPU (PFT_IPC_STAGED between processes), or any other rank
//    sharing this GPU (gpu_ranks > 1: N ranks per GPU, whose neighbours may sit on another GPU and
//    depend on a rank of ours): 32 blocks.  A thousand spinning blocks would leave no CU for a pair
//    kernel's workgroup (the whole register file of a CU) of the rank that raises the flag, which
//    then waits out PFT_IPC_TIMEOUT -- or, across two GPUs, closes a wait cycle through both;
//  - in the boundary pipeline (the wait beside an interior launch that does not wait for it): 128
//    blocks of 4 waves, 16 CUs' worth; the 20 MB of the receive still take ~10 us;
//  - otherwise (this rank alone on its GPU, waiting on the compute stream): up to 1024.
int pft_halo_wait_blocks(long n, int local_staged, int gpu_ranks, int on_boundary_stream)
{
  int blocks = (int)std::min<long>(1024, std::max<long>(1, (n + 255) / 256));
  if (local_staged || gpu_ranks > 1) blocks = std::min(blocks, 32);
  if (on_boundary_stream) blocks = std::min(blocks, 128);
  return blocks;
}

int pft_slab_set_gpu_ranks(pft_slab* s, int n)
{
  if (!s || n < 1) return -2;
  s->gpu_ranks = n;
  return 0;
}

int pft_flat_alloc(double** p, size_t n)
{
  HIPCHK(hipMalloc((void**)p, n * sizeof(double)));
  return 0;
}
int pft_flat_free(double* p)
{
  if (p) HIPCHK(hipFree(p));
  return 0;
}
int pft_flat_h2d(double* dst, const double* src, size_t n, void* stream)
{
  HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyHostToDevice, (hipStream_t)stream));
  return 0;
}
int pft_flat_d2h(double* dst, const double* src, size_t n, void* stream)
{
  HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, (hipStream_t)stream));
  return 0;
}
int pft_flat_combine(int stage, int n_chunks, const int* d_start, const int* d_size, const double* d_mult,
                     double coef, double h, const double* x, const double* k1, const double* k2, const double* k3,
                     const double* k4, const double* k5, double* out, double* d_eps2, void* stream)
{
  const int blocks = n_chunks < 4096 ? n_chunks : 4096;
  if (blocks <= 0) return -2;
  flat_combine_kernel<<<blocks, PFT_BLOCK, 0, (hipStream_t)stream>>>(
      stage, n_chunks, d_start, d_size, d_mult, coef, h, x, k1, k2, k3, k4, k5, out,
      (unsigned long long*)d_eps2, (unsigned int*)(d_eps2 + 1));
  HIPCHK(hipGetLastError());
  return 0;
}
int pft_stream_sync(void* stream)
{
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}
int pft_probe_copy(double* dst, const double* src, size_t n, void* stream)
{
  probe_copy_kernel<<<4096, 256, 0, (hipStream_t)stream>>>(dst, src, (long)n);
  HIPCHK(hipGetLastError());
  return 0;
}

int pft_dev_alloc(void** p, size_t bytes)
{
  HIPCHK(hipMalloc(p, bytes));
  return 0;
}
int pft_dev_free(void* p)
{
  if (p) HIPCHK(hipFree(p));
  return 0;
}
int pft_h2d(void* dst, const void* src, size_t bytes, void* stream)
{
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return 0;
}
int pft_memcpy_d2d_async(void* dst, const void* src, size_t bytes, void* stream)
{
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}
int pft_event_record_wait(void* from_stream, void* to_stream)
{
  hipEvent_t e;
  HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipEventRecord(e, (hipStream_t)from_stream));
  HIPCHK(hipStreamWaitEvent((hipStream_t)to_stream, e, 0));
  HIPCHK(hipEventDestroy(e));
  return 0;
}

}  // extern "C"
