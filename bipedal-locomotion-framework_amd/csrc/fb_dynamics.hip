// fb_dynamics.hip — FloatingBaseDynamicalSystem on the device.
//
// FloatingBaseSystemDynamics.cpp:102-251 takes the free-floating mass matrix M, the generalized
// bias forces h and the contact-frame Jacobians from iDynTree KinDynComputations and then solves
//   nu_dot = LLT(M [+ reg]) \ (-h + sum_c J_c^T w_c + [0; tau]).
// Here the rigid-body terms are computed directly, in the mixed representation (base velocity
// (dp_B/dt, w_B), world coordinates), for a kinematic tree of revolute joints, with spatial
// quantities taken about the WORLD ORIGIN, where a composite inertia is a plain sum:
//   link l:   spatial inertia I_l = (m, h = m c, Ibar = I_c + m(|c|^2 1 - c c^T)) (10 numbers),
//             spatial force   F_l = (tau_c + c x f, f),  f = m (a_c - g), tau_c = I_c al + w x I_c w
//             (accelerations at nu_dot = 0);
//   column:   motion axis S = (w, u): base linear e_a -> (0, e_a); base angular e_a -> (e_a, p_B x e_a);
//             joint j -> (z_j, o_j x z_j);
//   M_ij  = S_j^T (Ic_sub(i) S_i)  when column j acts on the subtree moved by column i (i >= j),
//   rhs_c = [tau] - S_c^T (sum of F_l over the subtree of c  -  contact wrenches on it, taken about
//           the origin),
// which is exactly sum_l m Jv^T Jv + Jw^T I Jw, h and J_c^T w_c of the Jacobian form
// (oracle/fb_dynamics.py evaluates that form; the two agree to rounding).
// One 64-lane workgroup (one wavefront) per system, everything in LDS:
//   1. per-joint rotations, lane per joint;  2. forward kinematics by pointer jumping along the
//   ancestor chains (every joint lane at once, log2 of the depth rounds);  3. per-link spatial inertia / force, lane per link;
//   4. contact wrenches, lane per contact;  5. subtree sums, lane per (subtree, parameter), the
//   ancestor bitmask of each link selecting the members;  6. column axes, their composite products
//   and the right-hand side, lane per column;  7. M, lane per lower-triangle entry;  8. Cholesky,
//   left-looking with one lane per row (one barrier per column);  9. forward and back
//   substitution with the right-hand side in registers (lane per row, pivots broadcast by
//   v_readlane, reciprocal pivots precomputed).
#include "blf_internal.h"
#include "contact_math.h"
#include "dcm_qp_common.h"   // the DPP prefix-scan levels (qp::tree_fwd / tree_has)
#include "fbk_math.h"

namespace blf {

#ifdef BLF_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of lane 0 for the first 64 systems.
__device__ unsigned long long g_fbd_stamps[12];
#define FSTAMP(t) unsigned long long t = __builtin_amdgcn_s_memtime()
#define FSTAMP_ADD(slot, t0) \
    do { if (blockIdx.x < 64 && threadIdx.x == 0) atomicAdd(&g_fbd_stamps[slot], __builtin_amdgcn_s_memtime() - (t0)); } while (0)
extern "C" int blf_debug_fbd_stamps(unsigned long long* out, int reset)
{
    unsigned long long h[12];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fbd_stamps), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < 12; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[12] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_fbd_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define FSTAMP(t)
#define FSTAMP_ADD(slot, t0)
#endif

namespace {

// Every kernel in this file runs one 64-lane wavefront per workgroup, and the LDS operations of a
// wavefront complete in program order, so lanes exchanging data through LDS need only a compiler
// barrier between the write and the read (no s_barrier, no full s_waitcnt).
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// link record: R 9 | p 3 | w 3 | v 3 | al 3 | a 3 | spatial inertia 10 (m, h, Ibar xx xy xz yy yz zz)
//              | spatial force 6 (tau_O, f)
// Per-lane records are read and written lane-strided (lane l at l * stride), so every stride is
// an ODD number of doubles: consecutive lanes then fall on distinct LDS bank pairs and an 8-byte
// access of 32 lanes is conflict-free.  With the even strides of the data sizes (40, 16, 12, 6
// doubles) SQ_LDS_BANK_CONFLICT was 83k quad-cycles per wave, 16 % of the Euler kernel's cycles
// (profiles/r03_fbd_euler_sq.json); BLF_FBD_PAD=0 builds the old layout for A/B.
#ifndef BLF_FBD_PAD
#define BLF_FBD_PAD 1
#endif
#ifndef BLF_FBD_CHOLB
#define BLF_FBD_CHOLB 2
#endif
// the Euler kernel's substitutions (fbd_eval FOLD): 0 two loops after the factorization, 1 the
// forward one inside it, 2 that and L stored column-major by the factorization itself.  Measured
// (profiles/r04_fbd_fold_ab.log, one c5 period of fbd_euler_kernel, two rounds on one box): 1 took
// 4.747 / 4.740 ms against 4.701 / 4.705 ms for 0 (the block's y broadcasts lengthen every
// factorization step's chain more than the separate loop costs); 2 spills 318 VGPRs.  So 0.
#ifndef BLF_FBD_SCANX   // the subtree sums' gathers: 1 = one ds_bpermute per component (0: three, A/B)
#define BLF_FBD_SCANX 1   // 4.657 / 4.640 against 4.671 / 4.656 ms per c5 period (profiles/r04_fbd_scanx_ab.log)
#endif
#ifndef BLF_FBD_LDSMODEL   // fbd_euler_kernel reads the model's constants from an LDS copy (A/B)
#define BLF_FBD_LDSMODEL 0   // 1: 5.92 / 5.93 against 4.24 / 4.24 ms per c5 period (profiles/r04_fbd_kinjump_ab.log)
#endif
#ifndef BLF_FBD_FOLD
#define BLF_FBD_FOLD 0
#endif
#ifndef BLF_FBD_PREFIX_LDS   // DFS subtree sums: step 5 leaves the prefix sums, step 6 takes the differences (1)
#define BLF_FBD_PREFIX_LDS 1   // or step 5 gathers them by lane shuffles (0, A/B): 3.812 / 3.811 against
                               // 4.077 / 4.074 ms per c5 period (profiles/r04_fbd_prefix_opq_ab.log)
#endif
#ifndef BLF_FBD_SUBST   // substitutions with the pivot scaling on the multipliers (1, A/B) or on the unknowns (0)
#define BLF_FBD_SUBST 0   // 1: 3.914 / 3.904 against 3.792 / 3.792 ms per c5 period (profiles/r04_fbd_subst_ab.log)
#endif
#ifndef BLF_FBD_KINJUMP   // steps 1-2 by pointer jumping (1) or tree level by level (0, A/B)
#define BLF_FBD_KINJUMP 1     // 4.238 / 4.239 against 4.688 / 4.704 ms per c5 period of fbd_euler_kernel
#endif                        // (profiles/r04_fbd_kinjump_ab.log); 15.3k -> 9.3k cycles per evaluation
#ifndef BLF_FBD_CSTAGE   // fbd_euler_kernel stages each system's contact / impedance constants in LDS (1) or
#define BLF_FBD_CSTAGE 1   // reads them from global memory every Euler step (0, A/B): 3.793 / 3.773 against
                           // 3.805 / 3.785 ms per c5 period (profiles/r04_cstage_asopq_ab.log)
#endif
#ifndef BLF_FBD_COLFIX   // the factorization's column sets at a compile-time stride (1, A/B) or at NV (0)
#define BLF_FBD_COLFIX 0   // 1: Cholesky 19.9k -> 14.8k cycles in fbd_dynamics_kernel, but one c5 period of the
#endif                     // Euler kernel 4.04 / 4.02 against 3.77 / 3.76 ms (profiles/r04_fbd_colfix_cstage_ab.log)
#ifndef BLF_FBD_OPQLANE   // fbd_eval's lane index opaque per evaluation (1) or not (0, A/B)
#define BLF_FBD_OPQLANE 1   // 3.812 / 3.811 against 3.856 / 3.860 ms per c5 period; SGPR spills 595 -> 366,
#endif                      // VGPR spills 17 -> 0 (profiles/r04_fbd_prefix_opq_ab.log)
#ifndef BLF_FBD_CSUB   // contact wrenches subtracted from the link forces in step 3 (1) or in step 5 (0, A/B)
#define BLF_FBD_CSUB 1  // 4.070 / 4.078 against 4.198 / 4.200 ms per c5 period (profiles/r04_fbd_csub_ab.log)
#endif

constexpr int kPad = BLF_FBD_PAD;
constexpr bool kPrefixLds = BLF_FBD_PREFIX_LDS && BLF_FBD_CSUB;   // (the base's contacts: step 3)
constexpr bool kSubst = BLF_FBD_SUBST && BLF_FBD_CHOLB > 1;        // (the pivots: the block factorization)
constexpr int kLinkRec = 40 + kPad;   // record stride (40 doubles of data)
constexpr int kR = 0, kP = 9, kW = 12, kV = 15, kAl = 18, kA = 21, kSI = 24, kSF = 34;
// The articulated-body layout (Smem aba): 27-double records.  Step 3 writes a link's spatial
// inertia / force over the first 16 doubles of its own record once it has read the kinematics
// (no other lane reads that record afterwards: the contacts, which do, run before step 3), and
// fbd_aba keeps joint j's slot (articulated inertia 21 | bias 6, later da 6) in link j + 1's record
// after reading that link's spatial terms.
constexpr int kLinkRecA = 27;
constexpr int kSIa = 0, kSFa = 10;
constexpr int kComp = 16;             // subtree sum: spatial inertia 10 | spatial force 6
constexpr int kCompS = kComp + kPad;  // its stride
constexpr int kCs = 16 + kPad;        // contact scratch: point 3 | wrench 6 | link 1 | spatial wrench 6
constexpr int kJrot = 12 + kPad;      // per-joint E_j Rot (9) | E_j a_j (3)
constexpr int kSax = 6 + kPad;        // column axis (w, u)

struct Smem {
    // one base pointer (per system: the two halves of a wavefront have their own) and wave-uniform
    // offsets, so the per-half base costs one address, not one per array
    double* base;
    int o_link, o_jrot, o_jz, o_jo, o_comp, o_sax, o_rhs, o_cscr, o_st, o_tq, o_anc, o_cst, o_imp;
    int ms;   // row stride of L (odd: the per-lane row accesses do not conflict)
    int lrec;   // link record stride: kLinkRec, or kLinkRecA for the articulated-body solve
    size_t total;
    // aba: the layout of the articulated-body solve (fbd_aba): records of kLinkRecA doubles that
    // later hold the spatial terms (kSIa / kSFa) and the joint slots, no subtree-sum / pivot-column
    // or column-axis arrays -- 9.3 KB per 30-DoF system instead of 19.2 KB, so two wavefronts of two
    // systems fit per SIMD
    __host__ __device__ Smem(double* b, int n, int C, bool aba = false) : base(b)
    {
        const int L = n + 1, NV = n + 6;
        ms = NV | 1;
        lrec = aba ? kLinkRecA : kLinkRec;
        size_t o = 0;
        auto take = [&](size_t k) {
            const int at = (int)o;
            o += (k + 1) & ~size_t(1);
            return at;
        };
        // link records; after the mass matrix is assembled the same space holds L (NV rows)
        const size_t lk = (size_t)lrec * L, lm = aba ? 0 : (size_t)NV * ms;
        o_link = take(lk > lm ? lk : lm);
        o_jrot = take(BLF_FBD_KINJUMP ? 0 : kJrot * (size_t)n);   // E_j Rot(a_j, s_j) (9) | E_j a_j (3): levels only
        o_jz = take(3 * (size_t)n);
        o_jo = take(3 * (size_t)n);
        // subtree sums [j] (joint j's subtree) and [n] (every link); later the pivot-column
        // buffers of the factorization (two sets of up to 4 columns, 8 NV)
        const size_t cp = (size_t)kCompS * (n + 1);
        const size_t cb = 8 * (size_t)(NV > 32 ? NV : 32);   // (BLF_FBD_COLFIX: 2 CB NVMAX)
        o_comp = take(aba ? 0 : cp > cb ? cp : cb);
        o_sax = take(aba ? 0 : kSax * (size_t)NV);
        o_rhs = take((size_t)NV);
        o_cscr = take((size_t)kCs * (C > 0 ? C : 1));
        o_st = take(18 + 2 * (size_t)n + (size_t)NV + 9);   // Euler state (6 + n + 3 + 9 + n) + acc + dR
        o_tq = take((size_t)n);                              // the joint impedance's torques
        o_anc = take((size_t)L);
        // fbd_euler_kernel's per-system constants (BLF_FBD_CSTAGE): each contact's link, frame
        // pose, null pose and parameters [C | 12 C | 12 C | 4 C]; the impedance's kp, kd, q_ref
        o_cst = take(BLF_FBD_CSTAGE ? 29 * (size_t)C : 0);
        o_imp = take(BLF_FBD_CSTAGE ? 3 * (size_t)n : 0);
        total = o;
    }
    __device__ __forceinline__ double* link() const { return base + o_link; }
    __device__ __forceinline__ double* jrot() const { return base + o_jrot; }
    __device__ __forceinline__ double* jz() const { return base + o_jz; }
    __device__ __forceinline__ double* jo() const { return base + o_jo; }
    __device__ __forceinline__ double* comp() const { return base + o_comp; }
    __device__ __forceinline__ double* sax() const { return base + o_sax; }
    __device__ __forceinline__ double* rhs() const { return base + o_rhs; }
    __device__ __forceinline__ double* cscr() const { return base + o_cscr; }
    __device__ __forceinline__ double* st() const { return base + o_st; }
    __device__ __forceinline__ double* tq() const { return base + o_tq; }
    __device__ __forceinline__ double* cst() const { return base + o_cst; }
    __device__ __forceinline__ double* imp() const { return base + o_imp; }
    __device__ __forceinline__ unsigned long long* anc() const
    {
        return reinterpret_cast<unsigned long long*>(base + o_anc);
    }
};

// doubles of fbd_euler_kernel's LDS model block (BLF_FBD_LDSMODEL)
template <int NVMAX>
__host__ __device__ constexpr int fbd_model_block()
{
    // rounded up to an even count: the halves' state blocks after it stay 16-B aligned
    return (3 * (NVMAX - 6) + 9 * (NVMAX - 6) + 3 * (NVMAX - 5) + 9 * (NVMAX - 5) + (NVMAX - 5) + 2 * (NVMAX - 6) +
            13 * BLF_FBD_MAX_CONTACTS + 1) & ~1;
}

struct Model {
    int n, F;
    const int32_t* parent;
    const double *jorig, *jrot, *jaxis, *mass, *com, *inertia, *fpose;
    const int32_t* flink;
    double g0, g1, g2, rho;
    const int32_t* jtype;   // [n] or nullptr: BLF_JOINT_PRISMATIC marks a sliding joint
    // fbd_euler_kernel's LDS copy (BLF_FBD_LDSMODEL): each contact's frame pose [C][12] and link
    // [C] (read through these when fbd_eval's LM is set)
    const double* cpose;
    const double* clink;
};

struct Contacts {
    int C;
    const int32_t* frame;
    const double* params;
    const double* null_pose;   // [B][C][12]
    const int32_t* law;        // [C] or null (every contact BLF_CONTACT_CONTINUOUS)
    const double* wrench;      // [B][C][6] the BLF_CONTACT_WRENCH contacts' wrenches
};

// Whether contact c applies the caller's wrench (BLF_CONTACT_WRENCH) instead of the
// ContinuousContactModel law
#ifndef BLF_FBD_LAWS   // 0: the continuous law only (A/B of the law branch, tools/gpu_r05i.sh)
#define BLF_FBD_LAWS 1
#endif
__device__ __forceinline__ bool given_wrench(const Contacts& ct, int c)
{
    return BLF_FBD_LAWS && ct.law != nullptr && ct.law[c] == BLF_CONTACT_WRENCH;
}

__device__ __forceinline__ void cross3(const double* a, const double* b, double* o)
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ double dot3(const double* a, const double* b)
{
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}

// sym 3x3 (xx xy xz yy yz zz) times vector
__device__ __forceinline__ void sym_mv(const double* I, const double* x, double* y)
{
    y[0] = (I[0] * x[0] + I[1] * x[1]) + I[2] * x[2];
    y[1] = (I[1] * x[0] + I[3] * x[1]) + I[4] * x[2];
    y[2] = (I[2] * x[0] + I[4] * x[1]) + I[5] * x[2];
}

__device__ __forceinline__ double bcast(double v, int src)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Systems per wavefront.  A model with NV = n + 6 <= 32 fits half a wavefront (lane hl < 32 owns
// joint / row hl), so one wavefront integrates two systems side by side, one per half (HW = 32
// lanes per system); larger models take the whole wavefront (HW = 64).  Every loop, mask and
// broadcast below is per half; both halves run the same model, so their control flow is the same.
template <int HW>
struct Half {
    int hl, half;   // lane within the system's half, and which half
    __device__ __forceinline__ Half() : hl(threadIdx.x & (HW - 1)), half(HW == 64 ? 0 : (int)threadIdx.x / HW) {}
    // a ballot restricted to this half (bit i = lane i of the half)
    __device__ __forceinline__ unsigned long long ballot(bool p) const
    {
        const unsigned long long b = __ballot(p);
        return HW == 64 ? b : (b >> (HW * half)) & ((1ull << HW) - 1);
    }
    // v of lane `src` of this half
    __device__ __forceinline__ int shfl(int v, int src) const { return __shfl(v, HW * half + src, kWave); }
    // v of lane k of this half, as a broadcast (v_readlane; two of them and a select for halves)
    __device__ __forceinline__ double bcast_k(double v, int k) const
    {
        if (HW == 64) return bcast(v, k);
        const double a = bcast(v, k), b = bcast(v, HW + k);
        return half ? b : a;
    }
};

// r[lane] of a register row (the diagonal entry of the lane's own row), compile-time indexed.
template <int NVMAX>
__device__ __forceinline__ double bcast_own_diag(const double* r, int lane)
{
    double d = 0.0;
#pragma unroll
    for (int k = 0; k < NVMAX; ++k)
        if (lane == k) d = r[k];
    return d;
}

// Tree topology, the same for every system and every Euler step: built once per workgroup.
// Lane j < n: joint j's parent link, origin, depth and child mask; anc[l] (LDS) every link's
// ancestor-joint mask.
struct Topo {
    int P, depth, maxdepth;
    double o0, o1, o2;
    unsigned long long cmask, bmask;
    int last;   // the last joint of joint lane's subtree (DFS preorder: the run [lane, last])
    int lastc;  // the same for column lane's joint (lane - 6; lanes < 6: 0)
    bool dfs;   // the joints are in DFS preorder (wave-uniform): every subtree is a contiguous run
};

template <int HW>
__device__ __forceinline__ Topo build_topo(const Model& m, const Smem& S)
{
    const Half<HW> H;
    const int n = m.n, lane = H.hl;
    const bool jl = lane < n;
    Topo t;
    t.P = jl ? m.parent[lane] : 0;
    t.o0 = jl ? m.jorig[3 * lane] : 0.0;
    t.o1 = jl ? m.jorig[3 * lane + 1] : 0.0;
    t.o2 = jl ? m.jorig[3 * lane + 2] : 0.0;
    // walk to the base through the parents held by the other lanes (joint Q - 1 moves link Q)
    unsigned long long an = jl ? 1ull << lane : 0ull;
    int depth = 0, Q = t.P;
    for (int it = 0; it < n; ++it) {
        const bool up = jl && Q > 0;
        if (!__ballot(up)) break;   // both halves hold the same model
        const int q = H.shfl(t.P, up ? Q - 1 : 0);
        if (up) {
            ++depth;
            an |= 1ull << (Q - 1);
            Q = q;
        }
    }
    t.depth = depth;
    if (jl) S.anc()[lane + 1] = an;
    if (lane == 0) S.anc()[0] = 0ull;
    t.cmask = 0ull;
    for (int j = 0; j < n; ++j) {
        const unsigned long long b = H.ballot(jl && t.P == j + 1);
        if (lane == j) t.cmask = b;
    }
    t.bmask = H.ballot(jl && t.P == 0);
    // DFS preorder: joint k attaches to the base or to a link on the path to link k (joint k - 1's
    // child), i.e. its parent link's joint is among joint k - 1's ancestors; then the subtree of
    // joint j is the run [j, j + size_j - 1], size_j = the joints whose ancestor masks hold j
    {
        const int src = lane > 0 ? lane - 1 : 0;
        const int lo = H.shfl((int)an, src), hi = H.shfl((int)(an >> 32), src);
        const unsigned long long prev = ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
        const bool ok = !jl || lane == 0 || t.P == 0 || ((prev >> (t.P - 1)) & 1ull);
        t.dfs = H.ballot(!ok) == 0ull;
        int size = 0;
        for (int j = 0; j < n; ++j) {
            const int c = __builtin_popcountll(H.ballot(jl && ((an >> j) & 1ull)));
            if (lane == j) size = c;
        }
        t.last = jl ? lane + size - 1 : 0;
        t.lastc = H.shfl(t.last, lane >= 6 && lane < n + 6 ? lane - 6 : 0);
    }
    int md = depth;
#pragma unroll
    for (int off = HW / 2; off >= 1; off >>= 1) {
        const int q = __shfl_xor(md, off, kWave);
        md = q > md ? q : md;
    }
    t.maxdepth = __builtin_amdgcn_readfirstlane(md);
    wave_sync();
    return t;
}

// Steps 1-2 of fbd_eval: per-joint rotations and forward kinematics (poses, mixed velocities,
// nu_dot = 0 accelerations) of every link into the link records.
// PRI: the model may hold prismatic joints (blf_fb_model.joint_type != NULL); the launchers
// instantiate the kernels both ways, so all-revolute models (config 5) pay nothing for it.
template <int HW, bool PRI>
__device__ __forceinline__ void fbd_kinematics_levels(const Model& m, const Smem& S, const double* bv,
                                                      const double* jvel, const double* bp, const double* bR,
                                                      const double* jp, const Topo& T)
{
    const int n = m.n;
    const int lane = Half<HW>().hl;
    const bool jl = lane < n;   // n <= 48 < 64: one joint per lane
    const int depth = T.depth, P = T.P, maxdepth = T.maxdepth;
    const double sd = jl ? jvel[lane] : 0.0;
    // 1. per-joint rotation E_j Rot(a_j, s_j) (Rodrigues) and E_j a_j, lane per joint
    if (jl) {
        const int j = lane;
        const double* a = m.jaxis + 3 * j;
        const double* E = m.jrot + 9 * j;
        double sn = 0.0, cs = 1.0;   // a prismatic joint does not rotate: E Rot(a, 0) = E exactly
        if (!(PRI && m.jtype[j] == BLF_JOINT_PRISMATIC)) sincos(jp[j], &sn, &cs);
        if (PRI && m.jtype[j] != BLF_JOINT_PRISMATIC && m.jtype[j] != BLF_JOINT_REVOLUTE)
            sn = cs = __builtin_nan("");   // an unknown joint type: the robot's outputs are NaN
        const double c1 = 1.0 - cs;
        const double K[9] = {0.0, -a[2], a[1], a[2], 0.0, -a[0], -a[1], a[0], 0.0};
        double Rr[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double K2 = (K[3 * r] * K[c] + K[3 * r + 1] * K[3 + c]) + K[3 * r + 2] * K[6 + c];
                Rr[3 * r + c] = ((r == c ? 1.0 : 0.0) + sn * K[3 * r + c]) + c1 * K2;
            }
        double* out = S.jrot() + kJrot * j;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int c = 0; c < 3; ++c)
                out[3 * r + c] = (E[3 * r] * Rr[c] + E[3 * r + 1] * Rr[3 + c]) + E[3 * r + 2] * Rr[6 + c];
            out[9 + r] = (E[3 * r] * a[0] + E[3 * r + 1] * a[1]) + E[3 * r + 2] * a[2];
        }
    }
    if (lane == 0) {
        double* b = S.link();
        for (int i = 0; i < 9; ++i) b[kR + i] = bR[i];
        for (int i = 0; i < 3; ++i) {
            b[kP + i] = bp[i]; b[kV + i] = bv[i]; b[kW + i] = bv[3 + i];
            b[kAl + i] = 0.0; b[kA + i] = 0.0;
        }
    }
    wave_sync();
    // 2. forward kinematics, one tree level at a time: poses, mixed velocities, nu_dot = 0
    //    accelerations of every joint whose parent link is done
    for (int lev = 0; lev <= maxdepth; ++lev) {
        if (jl && depth == lev) {
            const int j = lane;
            // the parent link's record and this joint's rotation into registers first (the child
            // record's stores could otherwise alias them and delay the loads)
            double pr[24], Ej[12];
            const double* prs = S.link() + S.lrec * P;
#pragma unroll
            for (int i = 0; i < 24; ++i) pr[i] = prs[i];
#pragma unroll
            for (int i = 0; i < 12; ++i) Ej[i] = S.jrot()[kJrot * j + i];
            const double o[3] = {T.o0, T.o1, T.o2};
            const double* RP = pr + kR;
            double cR[9], r[3], z[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    cR[3 * a + c] = (RP[3 * a] * Ej[c] + RP[3 * a + 1] * Ej[3 + c]) + RP[3 * a + 2] * Ej[6 + c];
                r[a] = (RP[3 * a] * o[0] + RP[3 * a + 1] * o[1]) + RP[3 * a + 2] * o[2];
                z[a] = (RP[3 * a] * Ej[9] + RP[3 * a + 1] * Ej[10]) + RP[3 * a + 2] * Ej[11];
            }
            const double zs[3] = {z[0] * sd, z[1] * sd, z[2] * sd};
            // prismatic (oracle/fb_dynamics.py): r = R_P o + z q, w_c = w_P, al_c = al_P,
            // v_c = v_P + w_P x r + z sd, a_c = a_P + al_P x r + w_P x (w_P x r) + 2 w_P x z sd
            const bool pri = PRI && m.jtype[j] == BLF_JOINT_PRISMATIC;
            if (pri) {
                const double qj = jp[j];
#pragma unroll
                for (int a = 0; a < 3; ++a) r[a] = r[a] + z[a] * qj;
            }
            double t1[3], t2[3], t3[3], t4[3];
            cross3(pr + kW, r, t1);            // w_P x r
            cross3(pr + kW, zs, t2);           // w_P x z sd
            cross3(pr + kAl, r, t3);           // al_P x r
            cross3(pr + kW, t1, t4);           // w_P x (w_P x r)
            double* cr = S.link() + S.lrec * (j + 1);
#pragma unroll
            for (int i = 0; i < 9; ++i) cr[kR + i] = cR[i];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const double pc = pr[kP + a] + r[a];
                cr[kP + a] = pc;
                S.jz()[3 * j + a] = z[a];
                S.jo()[3 * j + a] = pc;
                const double arev = (pr[kA + a] + t3[a]) + t4[a];
                cr[kW + a] = pri ? pr[kW + a] : pr[kW + a] + zs[a];
                cr[kV + a] = pri ? (pr[kV + a] + t1[a]) + zs[a] : pr[kV + a] + t1[a];
                cr[kAl + a] = pri ? pr[kAl + a] : pr[kAl + a] + t2[a];
                cr[kA + a] = pri ? arev + 2.0 * t2[a] : arev;
            }
        }
        wave_sync();
    }
}

// motion cross product (w, v) x (w2, v2) = (w x w2, w x v2 + v x w2), accumulated into o
__device__ __forceinline__ void crm_add(const double* s, const double* t, double* o)
{
    double a[3], b[3], c[3];
    cross3(s, t, a);
    cross3(s, t + 3, b);
    cross3(s + 3, t, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        o[i] = o[i] + a[i];
        o[3 + i] = o[3 + i] + (b[i] + c[i]);
    }
}

// Steps 1-2 by pointer jumping along the ancestor chains (BLF_FBD_KINJUMP): every joint lane runs
// at once, and a chain of depth D takes ceil(log2(D + 1)) rounds instead of D + 1 tree levels.
//  * Poses: lane j holds the transform (R, p) from link ptr (initially its parent; the base's
//    world pose is folded in at once where the parent is the base, ptr = 0 then means "anchored in
//    the world") to its link j + 1.  A round composes the record of link ptr -- the segment from
//    that link's own ptr -- in front: (R, p) <- (R_X R, p_X + R_X p), ptr <- ptr_X.
//  * Velocities and nu_dot = 0 accelerations as spatial vectors about the world origin: with the
//    joint motion U_k = qdot_k S_k (S_k = (z_k, o_k x z_k), prismatic (0, z_k)),
//      V_c = V_B + sum_{k in chain(c)} U_k,   A_c = A_B + V_B x s + sum_{i before k} U_i x U_k,
//    so the chain element (s, x) = (sum U, sum of the ordered cross products) composes as
//    (s_X + s_Y, x_X + x_Y + s_X x s_Y) -- the same jumping rounds.  The link records' mixed
//    quantities follow: w = V_w, v = V_v + w x p, al = A_w, a = A_v + al x p + w x v (V_B =
//    (w_B, v_B + p_B x w_B), A_B = (0, -(w_B x v_B)): the base's nu_dot = 0).
// A lane reads its partner's record before it writes its own in the same round: the wavefront's
// LDS operations complete in program order, so every read sees the previous round's values.
// Rounding differs from the level recursion (parity is the 1e-9 bar of the fb tests).
template <int HW, bool PRI>
__device__ __forceinline__ void fbd_kinematics_jump(const Model& m, const Smem& S, const double* bv,
                                                    const double* jvel, const double* bp, const double* bR,
                                                    const double* jp, const Topo& T)
{
    const Half<HW> H;
    const int n = m.n;
    const int lane = H.hl;
    const bool jl = lane < n;
    const int maxdepth = T.maxdepth;
    const double sd = jl ? jvel[lane] : 0.0;
    double Rb[9], pb[3], wb[3], vb[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) Rb[i] = bR[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        pb[i] = bp[i];
        vb[i] = bv[i];
        wb[i] = bv[3 + i];
    }
    if (lane == 0) {
        double* b = S.link();
        for (int i = 0; i < 9; ++i) b[kR + i] = Rb[i];
        for (int i = 0; i < 3; ++i) {
            b[kP + i] = pb[i]; b[kV + i] = vb[i]; b[kW + i] = wb[i];
            b[kAl + i] = 0.0; b[kA + i] = 0.0;
        }
    }
    // 1. the joint's own transform: E_j Rot(a_j, s_j) (Rodrigues) and the origin o_j (+ E_j a_j q)
    double R[9], p[3], ax[3];
    const bool pri = PRI && jl && m.jtype[lane] == BLF_JOINT_PRISMATIC;
    {
        const int j = jl ? lane : 0;
        const double* a = m.jaxis + 3 * j;
        const double* E = m.jrot + 9 * j;
        ax[0] = a[0]; ax[1] = a[1]; ax[2] = a[2];
        double sn = 0.0, cs = 1.0;
        if (jl && !pri) sincos(jp[j], &sn, &cs);
        if (PRI && jl && m.jtype[j] != BLF_JOINT_PRISMATIC && m.jtype[j] != BLF_JOINT_REVOLUTE)
            sn = cs = __builtin_nan("");   // an unknown joint type: the robot's outputs are NaN
        const double c1 = 1.0 - cs;
        const double K[9] = {0.0, -a[2], a[1], a[2], 0.0, -a[0], -a[1], a[0], 0.0};
        double Rr[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double K2 = (K[3 * r] * K[c] + K[3 * r + 1] * K[3 + c]) + K[3 * r + 2] * K[6 + c];
                Rr[3 * r + c] = ((r == c ? 1.0 : 0.0) + sn * K[3 * r + c]) + c1 * K2;
            }
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                R[3 * r + c] = (E[3 * r] * Rr[c] + E[3 * r + 1] * Rr[3 + c]) + E[3 * r + 2] * Rr[6 + c];
        p[0] = T.o0; p[1] = T.o1; p[2] = T.o2;
        if (pri) {
            const double qj = jp[j];
#pragma unroll
            for (int r = 0; r < 3; ++r)
                p[r] = p[r] + ((E[3 * r] * a[0] + E[3 * r + 1] * a[1]) + E[3 * r + 2] * a[2]) * qj;
        }
    }
    // the transform (RX, pX) in front of (R, p)
    auto compose = [&](const double* RX, const double* pX) {
        double Rn[9], pn[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int c = 0; c < 3; ++c)
                Rn[3 * r + c] = (RX[3 * r] * R[c] + RX[3 * r + 1] * R[3 + c]) + RX[3 * r + 2] * R[6 + c];
            pn[r] = pX[r] + ((RX[3 * r] * p[0] + RX[3 * r + 1] * p[1]) + RX[3 * r + 2] * p[2]);
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = Rn[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) p[i] = pn[i];
    };
    int ptr = jl ? T.P : 0;
    if (jl && ptr == 0) compose(Rb, pb);
    double* own = S.link() + S.lrec * (lane + 1);
    if (jl) {
#pragma unroll
        for (int i = 0; i < 9; ++i) own[kR + i] = R[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) own[kP + i] = p[i];
    }
    wave_sync();
    // 2a. poses: ceil(log2(maxdepth + 1)) rounds
    for (int span = 1; span <= maxdepth; span <<= 1) {
        const bool act = jl && ptr > 0;
        const int pn = H.shfl(ptr, act ? ptr - 1 : 0);
        if (act) {
            const double* x = S.link() + S.lrec * ptr;
            double RX[9], pX[3];
#pragma unroll
            for (int i = 0; i < 9; ++i) RX[i] = x[kR + i];
#pragma unroll
            for (int i = 0; i < 3; ++i) pX[i] = x[kP + i];
            compose(RX, pX);
#pragma unroll
            for (int i = 0; i < 9; ++i) own[kR + i] = R[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) own[kP + i] = p[i];
            ptr = pn;
        }
        wave_sync();
    }
    // 2b. the joint's world axis z = R_child a (Rot(a, s) a = a) and origin o = p_child; its motion
    double z[3], s[6], x[6];
#pragma unroll
    for (int r = 0; r < 3; ++r) z[r] = (R[3 * r] * ax[0] + R[3 * r + 1] * ax[1]) + R[3 * r + 2] * ax[2];
    {
        double oz[3];
        cross3(p, z, oz);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            s[i] = pri ? 0.0 : z[i] * sd;
            s[3 + i] = pri ? z[i] * sd : oz[i] * sd;
            x[i] = 0.0;
            x[3 + i] = 0.0;
        }
    }
    if (jl) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            S.jz()[3 * lane + a] = z[a];
            S.jo()[3 * lane + a] = p[a];
        }
        // the chain element in the record's w, v, al, a slots until the end
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            own[kW + i] = s[i];
            own[kAl + i] = x[i];
        }
    }
    wave_sync();
    // 2c. the chain sums: the same rounds
    ptr = jl ? T.P : 0;
    for (int span = 1; span <= maxdepth; span <<= 1) {
        const bool act = jl && ptr > 0;
        const int pn = H.shfl(ptr, act ? ptr - 1 : 0);
        if (act) {
            const double* e = S.link() + S.lrec * ptr;
            double sX[6], xX[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                sX[i] = e[kW + i];
                xX[i] = e[kAl + i];
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) x[i] = xX[i] + x[i];
            crm_add(sX, s, x);
#pragma unroll
            for (int i = 0; i < 6; ++i) s[i] = sX[i] + s[i];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                own[kW + i] = s[i];
                own[kAl + i] = x[i];
            }
            ptr = pn;
        }
        wave_sync();
    }
    // 2d. the records' mixed velocities and accelerations
    if (jl) {
        double VB[6], A[6], t[3];
        cross3(pb, wb, t);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            VB[i] = wb[i];
            VB[3 + i] = vb[i] + t[i];
        }
        cross3(wb, vb, t);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            A[i] = x[i];
            A[3 + i] = x[3 + i] - t[i];
        }
        crm_add(VB, s, A);
        double w[3], v[3], al[3], acc[3], u[3], q[3], r[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            w[i] = VB[i] + s[i];
            al[i] = A[i];
        }
        cross3(w, p, u);
#pragma unroll
        for (int i = 0; i < 3; ++i) v[i] = (VB[3 + i] + s[3 + i]) + u[i];
        cross3(al, p, q);
        cross3(w, v, r);
#pragma unroll
        for (int i = 0; i < 3; ++i) acc[i] = (A[3 + i] + q[i]) + r[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            own[kW + i] = w[i];
            own[kV + i] = v[i];
            own[kAl + i] = al[i];
            own[kA + i] = acc[i];
        }
    }
    wave_sync();
}


template <int HW, bool PRI>
__device__ __forceinline__ void fbd_kinematics(const Model& m, const Smem& S, const double* bv,
                                               const double* jvel, const double* bp, const double* bR,
                                               const double* jp, const Topo& T)
{
    if constexpr (BLF_FBD_KINJUMP) fbd_kinematics_jump<HW, PRI>(m, S, bv, jvel, bp, bR, jp, T);
    else fbd_kinematics_levels<HW, PRI>(m, S, bv, jvel, bp, bR, jp, T);
}

// ---- The articulated-body solve (round 5): nu_dot without M, its factorization or the
//      substitutions.  With every spatial quantity about the world origin no transform is needed
//      between a link and its parent, and the accelerations relative to nu_dot = 0 satisfy
//        da_c = da_p + s_j qdd_j   (joint j moves link c = j + 1 from its parent link p),
//        f_c  = F_c + I_c da_c     (F_c: step 3's force at nu_dot = 0, contacts subtracted),
//        s_j^T (sum of f over the subtree of c) = tau_j,
//      which the articulated inertias IA and biases pA solve in one inward and one outward sweep
//      over the tree levels (lane per joint):
//        IA_c = I_c + sum_children (IA_k - U_k U_k^T / D_k),  pA_c = F_c + sum_children (pA_k + U_k u_k / D_k),
//        U_j = IA_c s_j,  D_j = s_j^T U_j,  u_j = tau_j - s_j^T pA_c;
//        base: IA_0 da_0 = -pA_0 (6 x 6, every lane), qdd_B from da_0 = S_B qdd_B;
//        outward: qdd_j = (u_j - U_j^T da_p) / D_j,  da_c = da_p + s_j qdd_j.
//      The same solution as M nu_dot = rhs (Featherstone's ABA; the oracle's Jacobian form agrees
//      to rounding, tests/test_gpu_fb_dynamics.py at 1e-9 relative).  A model with a mass-matrix
//      regularisation (reg != NULL) keeps the factorization, which that term needs.
// 6 x 6 symmetric matrices as their upper triangle, row-major (21 entries).
__host__ __device__ constexpr int s6(int i, int j)
{
    return i <= j ? i * 6 - i * (i - 1) / 2 + (j - i) : j * 6 - j * (j - 1) / 2 + (i - j);
}

// the spatial inertia about the origin (m, h, Ibar xx xy xz yy yz zz) as a 6 x 6 on (w; u)
__device__ __forceinline__ void spatial6(const double* si, double (&I)[21])
{
    const double m = si[0], h0 = si[1], h1 = si[2], h2 = si[3];
    I[s6(0, 0)] = si[4]; I[s6(0, 1)] = si[5]; I[s6(0, 2)] = si[6];
    I[s6(1, 1)] = si[7]; I[s6(1, 2)] = si[8]; I[s6(2, 2)] = si[9];
    I[s6(0, 3)] = 0.0; I[s6(0, 4)] = -h2; I[s6(0, 5)] = h1;
    I[s6(1, 3)] = h2; I[s6(1, 4)] = 0.0; I[s6(1, 5)] = -h0;
    I[s6(2, 3)] = -h1; I[s6(2, 4)] = h0; I[s6(2, 5)] = 0.0;
    I[s6(3, 3)] = m; I[s6(3, 4)] = 0.0; I[s6(3, 5)] = 0.0;
    I[s6(4, 4)] = m; I[s6(4, 5)] = 0.0; I[s6(5, 5)] = m;
}

template <int HW, bool PRI>
__device__ __forceinline__ bool fbd_aba(const Model& m, const Smem& S, const double* tau, const double* bp,
                                        const Topo& T, int lane)
{
    const int n = m.n;
    const bool jl = lane < n;
    // joint j's slot: link j + 1's record (Smem aba), written after that link's spatial terms are read
    double* const rec = S.link();
    const int lr = S.lrec;
    bool ok = true;
    // this lane's joint axis s = (w; u) and torque
    double sv[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    double tq = 0.0;
    if (jl) {
        const double* z = S.jz() + 3 * lane;
        if (PRI && m.jtype[lane] == BLF_JOINT_PRISMATIC) {
            sv[3] = z[0]; sv[4] = z[1]; sv[5] = z[2];
        } else {
            sv[0] = z[0]; sv[1] = z[1]; sv[2] = z[2];
            cross3(S.jo() + 3 * lane, z, sv + 3);
        }
        tq = tau[lane];
    }
    double U[6], uD = 0.0, iD = 0.0;
#pragma unroll
    for (int a = 0; a < 6; ++a) U[a] = 0.0;
    // inward sweep, deepest joints first
    FSTAMP(a_in);
    for (int lev = T.maxdepth; lev >= 0; --lev) {
        if (jl && T.depth == lev) {
            const double* k = rec + lr * (lane + 1);
            double IA[21], pA[6];
            spatial6(k + kSIa, IA);
#pragma unroll
            for (int a = 0; a < 6; ++a) pA[a] = k[kSFa + a];
            for (unsigned long long b = T.cmask; b; b &= b - 1) {
                const double* c = rec + lr * (__builtin_ctzll(b) + 1);
#pragma unroll
                for (int e = 0; e < 21; ++e) IA[e] = IA[e] + c[e];
#pragma unroll
                for (int a = 0; a < 6; ++a) pA[a] = pA[a] + c[21 + a];
            }
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                double t = 0.0;
#pragma unroll
                for (int b = 0; b < 6; ++b) t = fma(IA[s6(a, b)], sv[b], t);
                U[a] = t;
            }
            double D = 0.0, sp = 0.0;
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                D = fma(sv[a], U[a], D);
                sp = fma(sv[a], pA[a], sp);
            }
            ok = ok && D > 0.0;
            iD = 1.0 / D;
            uD = (tq - sp) * iD;
            double* o = rec + lr * (lane + 1);
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double Ua = U[a] * iD;
#pragma unroll
                for (int b = a; b < 6; ++b) o[s6(a, b)] = fma(-Ua, U[b], IA[s6(a, b)]);
                o[21 + a] = fma(U[a], uD, pA[a]);
            }
        }
        wave_sync();
    }
    FSTAMP_ADD(4, a_in);
    // the base: IA_0 da_0 = -pA_0 (every lane, from the base's children's slots)
    FSTAMP(a_base);
    double da[6];
    {
        double IA[21], pA[6];
        const double* k = rec;
        spatial6(k + kSIa, IA);
#pragma unroll
        for (int a = 0; a < 6; ++a) pA[a] = k[kSFa + a];
        for (unsigned long long b = T.bmask; b; b &= b - 1) {
            const double* c = rec + lr * (__builtin_ctzll(b) + 1);
#pragma unroll
            for (int e = 0; e < 21; ++e) IA[e] = IA[e] + c[e];
#pragma unroll
            for (int a = 0; a < 6; ++a) pA[a] = pA[a] + c[21 + a];
        }
        // LDL^T of IA_0 in registers, then the two substitutions
        double L[21], d[6], x[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double dj = IA[s6(j, j)];
#pragma unroll
            for (int c = 0; c < j; ++c) dj = dj - (L[s6(j, c)] * L[s6(j, c)]) * d[c];
            ok = ok && dj > 0.0;
            d[j] = dj;
            const double idj = 1.0 / dj;
#pragma unroll
            for (int i = j + 1; i < 6; ++i) {
                double t = IA[s6(i, j)];
#pragma unroll
                for (int c = 0; c < j; ++c) t = t - (L[s6(i, c)] * L[s6(j, c)]) * d[c];
                L[s6(i, j)] = t * idj;
            }
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double t = -pA[i];
#pragma unroll
            for (int c = 0; c < i; ++c) t = t - L[s6(i, c)] * x[c];
            x[i] = t;
        }
#pragma unroll
        for (int i = 5; i >= 0; --i) {
            double t = x[i] / d[i];
#pragma unroll
            for (int c = i + 1; c < 6; ++c) t = t - L[s6(c, i)] * da[c];
            da[i] = t;
        }
    }
    FSTAMP_ADD(5, a_base);
    // outward sweep: qdd_j and the joint's child link's da, shallowest first
    FSTAMP(a_out);
    double qdd = 0.0;
    for (int lev = 0; lev <= T.maxdepth; ++lev) {
        if (jl && T.depth == lev) {
            double dp[6];
            const double* src = rec + lr * T.P;   // the parent joint's slot (T.P = 0: the base, unused)
#pragma unroll
            for (int a = 0; a < 6; ++a) dp[a] = T.P > 0 ? src[a] : da[a];
            double Ud = 0.0;
#pragma unroll
            for (int a = 0; a < 6; ++a) Ud = fma(U[a], dp[a], Ud);
            qdd = fma(-Ud, iD, uD);
            double* o = rec + lr * (lane + 1);
#pragma unroll
            for (int a = 0; a < 6; ++a) o[a] = fma(sv[a], qdd, dp[a]);
        }
        wave_sync();
    }
    // nu_dot: base (linear: da_0's u - p_B x w; angular: w), then the joints (p_B from the state:
    // the base record's position now holds its spatial force)
    const double* pB = bp;
    if (lane < 6) {
        const double w[3] = {da[0], da[1], da[2]};
        double pw[3];
        cross3(pB, w, pw);
        // (selects, not a lane-indexed array: that would live in scratch)
        const double lin = lane == 0 ? da[3] - pw[0] : lane == 1 ? da[4] - pw[1] : da[5] - pw[2];
        const double ang = lane == 3 ? da[0] : lane == 4 ? da[1] : da[2];
        S.rhs()[lane] = lane < 3 ? lin : ang;
    }
    if (jl) S.rhs()[6 + lane] = qdd;
    wave_sync();
    FSTAMP_ADD(6, a_out);
    const Half<HW> H;
    return H.ballot(!ok) == 0ull;
}

// World transform pose = (p, R row-major) and mixed twist tw = (v, w) of the frame whose pose in
// its link is fp, from the link's kinematics record k (the getWorldTransform / getFrameVel the
// reference hands each contact model, FloatingBaseSystemDynamics.cpp:225-226)
__device__ __forceinline__ void frame_state(const double* k, const double* fp, double* pose, double* tw)
{
    const double* R = k + kR;
    double d[3], t1[3];
    for (int a = 0; a < 3; ++a) {
        pose[a] = k[kP + a] + ((R[3 * a] * fp[0] + R[3 * a + 1] * fp[1]) + R[3 * a + 2] * fp[2]);
        for (int b = 0; b < 3; ++b)
            pose[3 + 3 * a + b] = (R[3 * a] * fp[3 + b] + R[3 * a + 1] * fp[6 + b]) + R[3 * a + 2] * fp[9 + b];
        d[a] = pose[a] - k[kP + a];
    }
    cross3(k + kW, d, t1);
    for (int a = 0; a < 3; ++a) {
        tw[a] = k[kV + a] + t1[a];
        tw[3 + a] = k[kW + a];
    }
}

// One evaluation of the dynamics for the system whose state sits in LDS (bv, jv, bp, bR, jp).
// Leaves the generalized acceleration in S.rhs() and returns false if the factorization failed.
// NVMAX >= n + 6 bounds the unrolled factorization loops (each lane keeps its row of M in
// registers).  Lane j < n owns joint j in steps 1, 2 and 5; lane i < NV owns row / column i in
// steps 6-9.
template <int NVMAX, int HW, bool PRI, int FOLD = 0, bool LM = false, bool CS = false, bool ABA = false>
__device__ __forceinline__ bool fbd_eval(const Model& m, const Smem& S, const double* bv,
                                         const double* jvel, const double* bp, const double* bR,
                                         const double* jp, const double* tau, const Contacts& ct,
                                         int64_t sys, const double* reg, const Topo& T)
{
    static_assert(NVMAX <= HW, "a system's rows must fit its lanes");
    const Half<HW> H;
    const int n = m.n, L = n + 1, NV = n + 6, MS = S.ms;
    // BLF_FBD_OPQLANE: the lane index made opaque once per evaluation, so the lane masks of the
    // unrolled loops (lane == k, lane > k, ...) are recomputed by one compare each instead of being
    // hoisted out of the Euler loop into SGPRs, which spill to VGPR lanes and reload by v_readlane
    int lane = H.hl;
    if constexpr (BLF_FBD_OPQLANE) asm volatile("" : "+v"(lane));
    const bool jl = lane < n;   // n <= 48 < 64: one joint per lane
    const int depth = T.depth, maxdepth = T.maxdepth;
    FSTAMP(f_t0);
    FSTAMP(f_t1);
    fbd_kinematics<HW, PRI>(m, S, bv, jvel, bp, bR, jp, T);
    FSTAMP_ADD(1, f_t1);
    FSTAMP(f_t2);
    // 3. per link: COM, world inertia, Newton-Euler force / moment, and the spatial inertia and
    //    force about the world origin (lane per link); BLF_FBD_CSUB: after step 4, with the
    //    contact wrenches on the link (about the origin) subtracted from its force here, once,
    //    instead of in every component group of the subtree sums
    auto link_step = [&]() {
    for (int l = lane; l < L; l += HW) {
        double* k = S.link() + S.lrec * l;
        const double* R = k + kR;
        const double* cl = m.com + 3 * l;
        const double* Ic = m.inertia + 9 * l;
        double rc[3], c[3];
        for (int a = 0; a < 3; ++a) {
            rc[a] = (R[3 * a] * cl[0] + R[3 * a + 1] * cl[1]) + R[3 * a + 2] * cl[2];
            c[a] = k[kP + a] + rc[a];
        }
        double RI[9];   // R Ic
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b)
                RI[3 * a + b] = (R[3 * a] * Ic[b] + R[3 * a + 1] * Ic[3 + b]) + R[3 * a + 2] * Ic[6 + b];
        const int ii[6] = {0, 0, 0, 1, 1, 2}, jj[6] = {0, 1, 2, 1, 2, 2};
        double Iw[6];
        for (int e = 0; e < 6; ++e) {
            const int a = ii[e], b = jj[e];
            Iw[e] = (RI[3 * a] * R[3 * b] + RI[3 * a + 1] * R[3 * b + 1]) + RI[3 * a + 2] * R[3 * b + 2];
        }
        double t1[3], t2[3], t3[3], f[3];
        cross3(k + kAl, rc, t1);
        cross3(k + kW, rc, t2);
        cross3(k + kW, t2, t3);
        const double ms = m.mass[l];
        const double g[3] = {m.g0, m.g1, m.g2};
        for (int a = 0; a < 3; ++a) f[a] = ms * (((k[kA + a] + t1[a]) + t3[a]) - g[a]);
        double Ia[3], Iwv[3], tq[3], cf[3];
        sym_mv(Iw, k + kAl, Ia);
        sym_mv(Iw, k + kW, Iwv);
        cross3(k + kW, Iwv, t1);
        for (int a = 0; a < 3; ++a) tq[a] = Ia[a] + t1[a];
        cross3(c, f, cf);
        const double cc = dot3(c, c);
        double* si = k + (ABA ? kSIa : kSI);   // (ABA: over the record's kinematics, read above)
        si[0] = ms;
        si[1] = ms * c[0]; si[2] = ms * c[1]; si[3] = ms * c[2];
        si[4] = Iw[0] + ms * (cc - c[0] * c[0]);
        si[5] = Iw[1] - ms * (c[0] * c[1]);
        si[6] = Iw[2] - ms * (c[0] * c[2]);
        si[7] = Iw[3] + ms * (cc - c[1] * c[1]);
        si[8] = Iw[4] - ms * (c[1] * c[2]);
        si[9] = Iw[5] + ms * (cc - c[2] * c[2]);
        double sfv[6];
        for (int a = 0; a < 3; ++a) {
            sfv[a] = tq[a] + cf[a];
            sfv[3 + a] = f[a];
        }
        if constexpr (BLF_FBD_CSUB) {
            for (int cc2 = 0; cc2 < ct.C; ++cc2) {   // branch-free: the loads do not wait for the test
                const double* sc = S.cscr() + kCs * cc2;
                const bool hit = (int)sc[9] == l;
                double w[6];
#pragma unroll
                for (int a = 0; a < 6; ++a) w[a] = sc[10 + a];
#pragma unroll
                for (int a = 0; a < 6; ++a) sfv[a] = hit ? sfv[a] - w[a] : sfv[a];
            }
        }
        double* sf = k + (ABA ? kSFa : kSF);
        for (int a = 0; a < 6; ++a) sf[a] = sfv[a];
    }
    };
    // 4. contacts: frame state + ContinuousContactModel wrench, and the wrench about the origin
    auto contacts_step = [&]() {
    for (int c = lane; c < ct.C; c += HW) {
        int l;
        const double* fp;
        if constexpr (CS) {
            l = (int)S.cst()[c];
            fp = S.cst() + ct.C + 12 * c;
        } else if constexpr (LM) {
            l = (int)m.clink[c];
            fp = m.cpose + 12 * c;
        } else {
            const int f = ct.frame[c];
            l = m.flink[f];
            fp = m.fpose + 12 * f;
        }
        double pose[12], tw[6];
        frame_state(S.link() + S.lrec * l, fp, pose, tw);
        double* sc = S.cscr() + kCs * c;
        if (given_wrench(ct, c)) {   // any ContactModel, evaluated by the caller
            const double* gw = ct.wrench + (sys * ct.C + c) * 6;
            for (int a = 0; a < 6; ++a) sc[3 + a] = gw[a];
        } else if constexpr (CS)
            contact_wrench(S.cst() + 25 * ct.C + 4 * c, tw, pose, S.cst() + 13 * ct.C + 12 * c, sc + 3);
        else
            contact_wrench(ct.params + 4 * c, tw, pose, ct.null_pose + (sys * ct.C + c) * 12, sc + 3);
        sc[0] = pose[0]; sc[1] = pose[1]; sc[2] = pose[2];
        sc[9] = (double)l;
        double xf[3];
        cross3(sc, sc + 3, xf);   // x_c x f_c
        for (int a = 0; a < 3; ++a) {
            sc[10 + a] = sc[6 + a] + xf[a];
            sc[13 + a] = sc[3 + a];
        }
    }
    wave_sync();
    };
    if constexpr (!BLF_FBD_CSUB) {
        link_step();
        FSTAMP_ADD(2, f_t2);
        FSTAMP(f_t3);
        contacts_step();
        FSTAMP_ADD(3, f_t3);
    } else {
        FSTAMP(f_t3);
        contacts_step();
        FSTAMP_ADD(3, f_t3);
        FSTAMP(f_t2b);
        link_step();
        wave_sync();
        FSTAMP_ADD(2, f_t2b);
    }
    static_assert(!ABA || BLF_FBD_CSUB, "the ABA layout needs the contacts before step 3");
    if constexpr (ABA) {   // steps 5-9 replaced by the articulated-body solve (no regularisation)
        FSTAMP(f_t4a);
        const bool ok = fbd_aba<HW, PRI>(m, S, tau, bp, T, lane);
        FSTAMP_ADD(7, f_t4a);
        FSTAMP_ADD(9, f_t0);
        return ok;
    }
    FSTAMP(f_t4);
    // 5. subtree sums of the spatial inertias and (link - contact) forces.  DFS-ordered models
    //    (every subtree a contiguous run of joints, T.dfs): one inclusive prefix sum over the
    //    joints' link terms per component, subtree_j = prefix[last_j] - prefix[j - 1], the base's
    //    = prefix[n - 1] + its own link terms: 5-6 shuffle levels instead of one LDS round trip
    //    and wave sync per tree level.  Other orders: level by level from the leaves up.
    if (T.dfs) {
        const int src = lane > 0 ? lane - 1 : 0;
        constexpr int G = 4;   // components per group (registers)
#pragma unroll
        for (int g = 0; g < kComp; g += G) {
            double v[G], pre[G];
            double bo[G];   // the base link's own terms (every lane reads them: no branch)
#pragma unroll
            for (int q = 0; q < G; ++q) {
                v[q] = jl ? S.link()[S.lrec * (lane + 1) + kSI + g + q] : 0.0;
                bo[q] = kPrefixLds ? 0.0 : S.link()[kSI + g + q];
            }
            if constexpr (!BLF_FBD_CSUB)
            for (int c = 0; c < ct.C; ++c) {
                const double* sc = S.cscr() + kCs * c;
                if (jl && (int)sc[9] == lane + 1)
#pragma unroll
                    for (int q = 0; q < G; ++q)
                        if (g + q >= 10) v[q] = v[q] - sc[g + q];
            }
#pragma unroll
            for (int q = 0; q < G; ++q) pre[q] = v[q];
            // inclusive prefix over the half's lanes by DPP (VALU moves, no LDS round trip): row
            // shifts 1, 2, 4, 8 inside each row of 16, then rows 1 / 3 add lane 15 of rows 0 / 2
            // (for HW = 64 also rows 2, 3 add lane 31) -- the QP kernels' forward tree levels
            const int wl = (int)threadIdx.x;
            auto level = [&](auto Lc) {
                constexpr int L = decltype(Lc)::value;
#pragma unroll
                for (int q = 0; q < G; ++q) {
                    const double t = qp::tree_fwd<L>(pre[q]);
                    if (qp::tree_has<L, true>(wl)) pre[q] = pre[q] + t;
                }
            };
            level(std::integral_constant<int, 0>{});
            level(std::integral_constant<int, 1>{});
            level(std::integral_constant<int, 2>{});
            level(std::integral_constant<int, 3>{});
            level(std::integral_constant<int, 4>{});
            if constexpr (HW == 64) level(std::integral_constant<int, 5>{});
            if constexpr (kPrefixLds) {   // step 6 takes prefix[last_j] - prefix[j - 1] itself
#pragma unroll
                for (int q = 0; q < G; ++q)
                    if (jl) S.comp()[kCompS * lane + g + q] = pre[q];
                (void)bo;
                (void)src;
                continue;
            }
#pragma unroll
            for (int q = 0; q < G; ++q) {
#if BLF_FBD_SCANX
                // the previous lane's prefix by a DPP wavefront rotation (a half's lane 0 does not
                // use it) and the total by v_readlane: one ds_bpermute per component, not three
                const double atl = __shfl(pre[q], T.last, HW);
                const double bef = qp::dpp1<qp::kPrevWrap>(pre[q]);
                const double tot = H.bcast_k(pre[q], n - 1);
                (void)src;
#else
                const double atl = __shfl(pre[q], T.last, HW);
                const double bef = __shfl(pre[q], src, HW);
                const double tot = __shfl(pre[q], n - 1, HW);
#endif
                if (jl) S.comp()[kCompS * lane + g + q] = lane > 0 ? atl - bef : atl;
                if constexpr (BLF_FBD_CSUB) {
                    const double b = bo[q] + tot;
                    if (lane == 0) S.comp()[kCompS * n + g + q] = b;
                } else if (lane == 0) {
                    double b = bo[q] + tot;
                    for (int c = 0; c < ct.C; ++c) {
                        const double* sc = S.cscr() + kCs * c;
                        if (g + q >= 10 && (int)sc[9] == 0) b = b - sc[g + q];
                    }
                    S.comp()[kCompS * n + g + q] = b;
                }
            }
        }
        wave_sync();
    } else
    for (int lev = maxdepth; lev >= -1; --lev) {
        const bool mine = lev >= 0 ? (jl && depth == lev) : lane == 0;
        if (mine) {
            const int l = lev >= 0 ? lane + 1 : 0;               // the subtree's root link
            const unsigned long long ch = lev >= 0 ? T.cmask : T.bmask;
            double acc[kComp];
#pragma unroll
            for (int p = 0; p < kComp; ++p) acc[p] = S.link()[S.lrec * l + kSI + p];
            if constexpr (!BLF_FBD_CSUB)
            for (int c = 0; c < ct.C; ++c) {
                const double* sc = S.cscr() + kCs * c;
                if ((int)sc[9] == l)
#pragma unroll
                    for (int p = 10; p < kComp; ++p) acc[p] = acc[p] - sc[p];
            }
            for (unsigned long long b = ch; b; b &= b - 1) {
                const double* cs = S.comp() + kCompS * __builtin_ctzll(b);
#pragma unroll
                for (int p = 0; p < kComp; ++p) acc[p] = acc[p] + cs[p];
            }
            double* dst = S.comp() + kCompS * (lev >= 0 ? lane : n);
#pragma unroll
            for (int p = 0; p < kComp; ++p) dst[p] = acc[p];
        }
        wave_sync();
    }
    FSTAMP_ADD(4, f_t4);
    FSTAMP(f_t5);
    // 6. lane c: column axis S_c = (w, u) (to LDS), F_c = Ic S_c with Ic the subtree sum the
    //    column moves (registers), rhs_c = [tau] - S_c^T (subtree force)
    const double* pB = S.link() + kP;
    double y = 0.0, Fc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (lane < NV) {
        const int c = lane;
        double w[3] = {0.0, 0.0, 0.0}, u[3] = {0.0, 0.0, 0.0};
        if (c < 3) {
            u[c] = 1.0;
        } else if (c < 6) {
            w[c - 3] = 1.0;
            cross3(pB, w, u);
        } else {
            const int j = c - 6;
            if (PRI && m.jtype[j] == BLF_JOINT_PRISMATIC) {   // S = (0; z): a pure translation
                for (int a = 0; a < 3; ++a) u[a] = S.jz()[3 * j + a];
            } else {
                for (int a = 0; a < 3; ++a) w[a] = S.jz()[3 * j + a];
                cross3(S.jo() + 3 * j, w, u);
            }
        }
        double Iv[kComp];
        if (kPrefixLds && T.dfs) {   // the subtree sums from the prefix sums step 5 left
            const int j = c - 6;
            const double* hp = S.comp() + kCompS * (c < 6 ? n - 1 : T.lastc);
            const double* lp = c < 6 ? S.link() + kSI : S.comp() + kCompS * (j > 0 ? j - 1 : 0);
#pragma unroll
            for (int p = 0; p < kComp; ++p) {
                const double h = hp[p], l = lp[p];
                Iv[p] = c < 6 ? l + h : (j > 0 ? h - l : h);
            }
        } else {
#pragma unroll
            for (int p = 0; p < kComp; ++p) Iv[p] = S.comp()[kCompS * (c < 6 ? n : c - 6) + p];
        }
        const double* I = Iv;
        double Iwv[3], hu[3], wh[3];
        sym_mv(I + 4, w, Iwv);
        cross3(I + 1, u, hu);
        cross3(w, I + 1, wh);
        double* sa = S.sax() + kSax * c;
        for (int a = 0; a < 3; ++a) {
            sa[a] = w[a];
            sa[3 + a] = u[a];
            Fc[a] = Iwv[a] + hu[a];
            Fc[3 + a] = wh[a] + I[0] * u[a];
        }
        y = (c >= 6 ? tau[c - 6] : 0.0) - (dot3(w, I + 10) + dot3(u, I + 13));
    }
    const unsigned long long myanc = (lane >= 6 && lane < NV) ? S.anc()[lane - 5] : 0ull;
    wave_sync();
    FSTAMP_ADD(5, f_t5);
    FSTAMP(f_t6);
    // 7. row i of M in registers: M_ij = S_j . F_i when column j moves the subtree of column i
    //    (j < 6, or joint j - 6 an ancestor of column i's link)
    // (no branch per column: a branch between an LDS read and its use serialises the reads; an
    // index past the last column is clamped and its value discarded by the row predicate)
    double r[NVMAX];
#pragma unroll
    for (int j = 0; j < NVMAX; ++j) {
        const double* sa = S.sax() + kSax * (j < NV ? j : NV - 1);   // every lane reads the same S_j
        const double v = dot3(sa, Fc) + dot3(sa + 3, Fc + 3);
        const bool vis = j <= lane && lane < NV && (j < 6 || ((myanc >> (j - 6)) & 1ull));
        r[j] = vis ? v : 0.0;
    }
    if (reg && lane < NV)
#pragma unroll
        for (int j = 0; j < NVMAX; ++j)
            if (j < NV && j <= lane) r[j] = r[j] + reg[NV * lane + j];
    FSTAMP_ADD(6, f_t6);
    FSTAMP(f_t7);
    // 8. Cholesky M = L L^T, right-looking, lane i keeps row i in registers, CB columns per step
    //    (BLF_FBD_CHOLB; 1: one column per step): every lane factors the step's CB x CB diagonal
    //    block from its broadcast entries (rows past the matrix: identity), computes its own CB
    //    entries by the same forward substitution (so a lane inside the block reproduces the
    //    block's row bit for bit), and the CB columns of the rows below go through one LDS buffer
    //    set (two sets, alternating) and are read back as broadcasts: one LDS round trip per CB
    //    pivots, where the dependent chain of pivot, column store and read-back is the
    //    Cholesky's time at one wavefront per SIMD
    bool ok = true;
#if BLF_FBD_CHOLB > 1
    // the block must divide the register row (NVMAX = 54 for the largest model: 2)
    constexpr int CB = NVMAX % BLF_FBD_CHOLB == 0 ? BLF_FBD_CHOLB : 2;
    static_assert(NVMAX % CB == 0, "block size divides the register row");
    // FOLD >= 1: the forward substitution L z = y rides along: every lane also solves the block's
    // CB unknowns z_{k..k+CB-1} from the broadcast y entries of the block's lanes, the block's
    // lanes keep theirs, the rows below subtract L_{lane,k+i} z_{k+i}: no separate loop of NV
    // dependent broadcasts.  FOLD == 2: the columns also go to their final place, L column-major
    // over the dead link records (Lm[MS c + row], odd MS), which the back substitution then reads
    // lane-strided, instead of a separate row-major store of L.
    double* Lm = S.link();
#pragma unroll
    for (int k = 0; k < NVMAX; k += CB) {
        if (k < NV) {
            double Lb[CB][CB], il[CB];
#pragma unroll
            for (int i = 0; i < CB; ++i) {
                const bool in = k + i < NV;
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    double t = in ? H.bcast_k(r[k + j], k + i) : 0.0;   // M_{k+i,k+j}
#pragma unroll
                    for (int c = 0; c < j; ++c) t = t - Lb[i][c] * Lb[j][c];
                    Lb[i][j] = t * il[j];
                }
                double d = in ? H.bcast_k(r[k + i], k + i) : 1.0;       // M_{k+i,k+i}
#pragma unroll
                for (int c = 0; c < i; ++c) d = d - Lb[i][c] * Lb[i][c];
                ok = ok && (d > 0.0);
                // 1 / sqrt: v_rsq_f64 and one Newton step (parity with the oracle is at 1e-9)
                double q = __builtin_amdgcn_rsq(d);
                il[i] = q * (1.5 - (0.5 * d) * (q * q));
                Lb[i][i] = d * il[i];
                // 1 / L_kk for the substitutions (BLF_FBD_SUBST); S.rhs() is free until the end
                if (kSubst && HW == 32 && lane == 0 && k + i < NV) S.rhs()[k + i] = il[i];
            }
            // this lane's entries L_{lane,k..k+CB-1} (upper-triangle junk inside the block, unread)
            double li[CB];
#pragma unroll
            for (int i = 0; i < CB; ++i) {
                double t = r[k + i];
#pragma unroll
                for (int c = 0; c < i; ++c) t = t - li[c] * Lb[i][c];
                li[i] = t * il[i];
            }
            if constexpr (FOLD >= 1) {
            double z[CB];
#pragma unroll
            for (int i = 0; i < CB; ++i) {
                double t = k + i < NV ? H.bcast_k(y, k + i) : 0.0;
#pragma unroll
                for (int c = 0; c < i; ++c) t = t - Lb[i][c] * z[c];
                z[i] = t * il[i];
            }
            double yl = y;
#pragma unroll
            for (int i = 0; i < CB; ++i) yl = yl - li[i] * z[i];
#pragma unroll
            for (int i = 0; i < CB; ++i) y = lane == k + i ? z[i] : y;
            y = lane >= k + CB ? yl : y;
            }
            // BLF_FBD_COLFIX: the column sets at the compile-time stride NVMAX, every lane of the
            // rows (padding lanes: zeros) writing its entry, so the update reads every row at a
            // constant offset (no clamped per-row address registers; paired LDS reads)
            constexpr int kColS = BLF_FBD_COLFIX ? NVMAX : 0;
            double* col = FOLD >= 2 ? Lm + MS * k
                                    : S.comp() + ((k / CB) & 1) * CB * (BLF_FBD_COLFIX ? NVMAX : NV);
            const int cst = FOLD >= 2 ? MS : (BLF_FBD_COLFIX ? kColS : NV);
#define FBD_COL(i, row) col[(i) * cst + (row)]
#pragma unroll
            for (int i = 0; i < CB; ++i) {
                r[k + i] = lane >= k ? li[i] : r[k + i];
                if ((BLF_FBD_COLFIX && FOLD < 2 ? lane < NVMAX : lane < NV) && k + i < NV) FBD_COL(i, lane) = r[k + i];
            }
            wave_sync();
            // no row predicate (as below): lanes above row j update only upper-triangle entries
#pragma unroll
            for (int j = k + CB; j < NVMAX; ++j) {
                const int jj = (BLF_FBD_COLFIX && FOLD < 2) ? j : (j < NV ? j : NV - 1);
                double t = r[j];
#pragma unroll
                for (int i = CB - 1; i >= 0; --i) t = fma(-r[k + i], FBD_COL(i, jj), t);
                r[j] = t;
            }
#undef FBD_COL
        }
    }
#else
    // 8. Cholesky M = L L^T, right-looking, lane i keeps row i in registers; column k of the
    //    rows below the pivot goes through an LDS buffer (two, alternating) and is read back as
    //    broadcasts
#pragma unroll
    for (int k = 0; k < NVMAX; ++k) {
        if (k < NV) {
            const double piv = H.bcast_k(r[k], k);
            ok = ok && (piv > 0.0);
            // 1 / sqrt(piv): v_rsq_f64 and one Newton step (the factorization's accuracy is that
            // of its rounding errors; parity with the oracle is at 1e-9)
            double isq = __builtin_amdgcn_rsq(piv);
            isq = isq * (1.5 - (0.5 * piv) * (isq * isq));
            r[k] = lane == k ? piv * isq : (lane > k ? r[k] * isq : r[k]);
            double* col = S.comp() + (k & 1) * NV;
            if (lane < NV) col[lane] = r[k];
            wave_sync();
            // No row predicate: a lane above row j only updates its upper-triangle entry r[j],
            // which nothing reads (pivots are diagonal, the substitutions and the stored L use
            // j <= lane), so the update is one LDS broadcast read and one fma per entry.  j >= NV
            // touches only lanes past the matrix.
#pragma unroll
            for (int j = k + 1; j < NVMAX; ++j) {
                const double ljk = col[j < NV ? j : NV - 1];
                r[j] = fma(-r[k], ljk, r[j]);   // parity here is 1e-9 relative, not bitwise
            }
        }
    }
#endif
    FSTAMP_ADD(7, f_t7);
    FSTAMP(f_t8);
#if BLF_FBD_CHOLB > 1
    if constexpr (FOLD == 1) {
    // 9. L z = y is done (folded into the factorization); L^T x = z with row k of L read from
    //    LDS (the link records are dead by now), one step ahead
    const double idg = lane < NV ? 1.0 / bcast_own_diag<NVMAX>(r, lane) : 0.0;
    if (lane < NV)
#pragma unroll
        for (int j = 0; j < NVMAX; ++j)
            if (j < NV && j <= lane) Lm[MS * lane + j] = r[j];
    wave_sync();
    double lki = (lane < NV - 1) ? Lm[MS * (NV - 1) + lane] : 0.0;
    for (int k = NV - 1; k >= 0; --k) {
        const double lnext = (k > 0 && lane < k - 1) ? Lm[MS * (k - 1) + lane] : 0.0;   // read ahead
        if (lane == k) y = y * idg;
        const double xk = H.bcast_k(y, k);
        if (lane < k) y = y - lki * xk;
        lki = lnext;
    }
    } else if constexpr (FOLD >= 2) {
    // 9. L z = y is done (folded into the factorization); L^T x = z with L's row k read from the
    //    column-major L (Lm[MS lane + k] = L_{k,lane}, lane-strided, one step ahead); lane k
    //    scales its own entry, one broadcast per step
    const double idg = lane < NV ? 1.0 / bcast_own_diag<NVMAX>(r, lane) : 0.0;
    double lki = (lane < NV - 1) ? Lm[MS * lane + (NV - 1)] : 0.0;
    for (int k = NV - 1; k >= 0; --k) {
        const double lnext = (k > 0 && lane < k - 1) ? Lm[MS * lane + (k - 1)] : 0.0;   // read ahead
        if (lane == k) y = y * idg;
        const double xk = H.bcast_k(y, k);
        if (lane < k) y = y - lki * xk;
        lki = lnext;
    }
    } else {
#endif
    // 9. L z = y with the rows in registers, then L^T x = z with row k of L read from LDS (the
    //    link records are dead by now); lane k scales its own entry, one broadcast per step.  Two
    //    unknowns per step (the 2 x 2 block solved by every lane, as in the factorization) measured
    //    the same: 6.054 / 6.069 against 6.081 / 6.073 ms per c5 period of the Euler kernel
    if constexpr (kSubst && HW == 32) {
    // BLF_FBD_SUBST (two systems per wavefront; LLVM's register allocator crashes on it in the
    // one-system instantiations): the unknown's scaling rides on the multiplier, not on the broadcast value:
    // step k broadcasts lane k's unscaled entry t_k and the rows update y_i -= (L_ik / L_kk) t_k,
    // whose factor is known ahead; the pivots 1 / L_kk come from the factorization (S.rhs()), and
    // every entry is scaled once at the end.  Per step the dependent chain is the broadcast and
    // one fma (was: scale, select, broadcast, multiply, subtract).
    const double* ilv = S.rhs();
    const double idg = lane < NV ? ilv[lane] : 0.0;
    double ilk = ilv[0];
#pragma unroll
    for (int k = 0; k < NVMAX; ++k) {   // k >= NV changes only lanes past the matrix
        const double ilnext = ilv[k + 1 < NV ? k + 1 : NV - 1];   // read ahead
        const double t = H.bcast_k(y, k);
        const double f = lane > k ? r[k] * ilk : 0.0;
        y = fma(-f, t, y);
        ilk = ilnext;
    }
    y = y * idg;
    double* Lr = S.link();
    if (lane < NV)
#pragma unroll
        for (int j = 0; j < NVMAX; ++j)
            if (j < NV && j <= lane) Lr[MS * lane + j] = r[j];
    wave_sync();
    double lki = (lane < NV - 1) ? Lr[MS * (NV - 1) + lane] : 0.0;
    ilk = ilv[NV - 1];
    for (int k = NV - 1; k >= 0; --k) {
        const double lnext = (k > 0 && lane < k - 1) ? Lr[MS * (k - 1) + lane] : 0.0;   // read ahead
        const double ilnext = ilv[k > 0 ? k - 1 : 0];
        const double t = H.bcast_k(y, k);
        const double f = lane < k ? lki * ilk : 0.0;
        y = fma(-f, t, y);
        lki = lnext;
        ilk = ilnext;
    }
    y = y * idg;
    } else {
    const double idg = lane < NV ? 1.0 / bcast_own_diag<NVMAX>(r, lane) : 0.0;
#pragma unroll
    for (int k = 0; k < NVMAX; ++k) {   // k >= NV changes only lanes past the matrix
        y = lane == k ? y * idg : y;
        const double xk = H.bcast_k(y, k);
        const double f = lane > k ? r[k] : 0.0;
        y = y - f * xk;
    }
    double* Lr = S.link();
    if (lane < NV)
#pragma unroll
        for (int j = 0; j < NVMAX; ++j)
            if (j < NV && j <= lane) Lr[MS * lane + j] = r[j];
    wave_sync();
    double lki = (lane < NV - 1) ? Lr[MS * (NV - 1) + lane] : 0.0;
    for (int k = NV - 1; k >= 0; --k) {
        const double lnext = (k > 0 && lane < k - 1) ? Lr[MS * (k - 1) + lane] : 0.0;   // read ahead
        if (lane == k) y = y * idg;
        const double xk = H.bcast_k(y, k);
        if (lane < k) y = y - lki * xk;
        lki = lnext;
    }
    }
#if BLF_FBD_CHOLB > 1
    }
#endif
    if (lane < NV) S.rhs()[lane] = y;
    wave_sync();
    FSTAMP_ADD(8, f_t8);
    FSTAMP_ADD(9, f_t0);
    return ok;
}

template <int NVMAX, int HW, bool PRI, bool ABA>
__global__ __launch_bounds__(64) void fbd_dynamics_kernel(Model m, blf_fb_state st,
                                                          const double* __restrict__ tau,
                                                          Contacts ct, const double* reg,
                                                          blf_fb_state out, int64_t batch)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const Half<HW> H;
    const int n = m.n, NV = n + 6;
    const Smem S(smem + H.half * Smem(nullptr, n, ct.C, ABA).total, n, ct.C, ABA);
    // system of this half; a missing second system of the last wavefront recomputes the last one
    // and writes nothing
    const int64_t q0 = (int64_t)blockIdx.x * (kWave / HW) + H.half;
    const bool active = q0 < batch;
    const int64_t q = active ? q0 : batch - 1;
    const int lane = H.hl;
    double* loc = S.st();   // bv 6 | jv n | bp 3 | bR 9 | jp n
    for (int i = lane; i < 18 + 2 * n; i += HW) {
        double v;
        if (i < 6) v = st.base_vel[6 * q + i];
        else if (i < 6 + n) v = st.joint_vel[(int64_t)n * q + (i - 6)];
        else if (i < 9 + n) v = st.base_pos[3 * q + (i - 6 - n)];
        else if (i < 18 + n) v = st.base_rot[9 * q + (i - 9 - n)];
        else v = st.joint_pos[(int64_t)n * q + (i - 18 - n)];
        loc[i] = v;
    }
    wave_sync();
    const Topo T = build_topo<HW>(m, S);
    const bool ok = fbd_eval<NVMAX, HW, PRI, 0, false, false, ABA>(m, S, loc, loc + 6, loc + 6 + n, loc + 9 + n, loc + 18 + n,
                                        tau + (int64_t)n * q, ct, q, reg, T);
    if (!active) return;
    const double nan = __builtin_nan("");
    for (int c = lane; c < NV; c += HW) {
        const double a = ok ? S.rhs()[c] : nan;
        if (c < 6) out.base_vel[6 * q + c] = a;
        else out.joint_vel[(int64_t)n * q + (c - 6)] = a;
    }
    if (lane == 0) {
        double dR[9];
        fbk_rot_rate(m.rho, loc + 9 + n, loc + 3, dR);
        for (int i = 0; i < 3; ++i) out.base_pos[3 * q + i] = loc[i];
        for (int i = 0; i < 9; ++i) out.base_rot[9 * q + i] = dR[i];
    }
    for (int j = lane; j < n; j += HW) out.joint_pos[(int64_t)n * q + j] = loc[6 + j];
}

// The joint impedance of blf_fbd_euler_integrate_impedance: tau = kp (q_ref - q) - kd qdot, set as
// the control input before every Euler step (kp == nullptr: the constant torques `tau`).
struct Impedance {
    const double *kp, *kd, *qref;
};

template <int NVMAX, int HW, bool PRI, bool ABA>
// Two systems per wavefront (HW = 32) keep more state live per wave: capping it at 256 VGPRs for
// two waves per SIMD spills (9.40 ms per c5 period), one wave per SIMD does not (8.29 ms, against
// 9.29 ms with one system per wavefront at two waves per SIMD; tools/ab_c5.sh).
__global__ __launch_bounds__(64, HW == 32 ? 1 : 2) void fbd_euler_kernel(Model m, blf_fb_state st,
                                                          const double* __restrict__ tau,
                                                          Contacts ct, const double* reg,
                                                          int32_t nsteps, double dT, double dT_last,
                                                          Impedance imp, int64_t batch)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const Half<HW> H;
    const int n = m.n, NV = n + 6;
    // BLF_FBD_LDSMODEL (two systems per wavefront): the model's per-joint / per-link constants,
    // the gains and the contacts' frames copied once into a block at the start of LDS, at
    // compile-time offsets, so the Euler loop reads them from LDS and holds no pointers to them
    constexpr bool kLM = BLF_FBD_LDSMODEL && HW == 32;
    constexpr bool kCS = BLF_FBD_CSTAGE && !kLM && HW == 32;   // (LLVM's allocator crashes on the HW = 64 form)
    constexpr int kMB = kLM ? fbd_model_block<NVMAX>() : 0;
    const Smem S(smem + kMB + H.half * Smem(nullptr, n, ct.C, ABA).total, n, ct.C, ABA);
    const int lane = H.hl;
    if constexpr (kLM) {
        constexpr int J = NVMAX - 6, Lk = NVMAX - 5;
        constexpr int oA = 0, oR = oA + 3 * J, oC = oR + 9 * J, oI = oC + 3 * Lk, oM = oI + 9 * Lk;
        constexpr int oKp = oM + Lk, oKd = oKp + J, oP = oKd + J, oL = oP + 12 * BLF_FBD_MAX_CONTACTS;
        const int t = threadIdx.x, L = n + 1;
        for (int i = t; i < 3 * n; i += kWave) smem[oA + i] = m.jaxis[i];
        for (int i = t; i < 9 * n; i += kWave) smem[oR + i] = m.jrot[i];
        for (int i = t; i < 3 * L; i += kWave) smem[oC + i] = m.com[i];
        for (int i = t; i < 9 * L; i += kWave) smem[oI + i] = m.inertia[i];
        for (int i = t; i < L; i += kWave) smem[oM + i] = m.mass[i];
        if (imp.kp)
            for (int i = t; i < n; i += kWave) {
                smem[oKp + i] = imp.kp[i];
                smem[oKd + i] = imp.kd[i];
            }
        for (int i = t; i < 12 * ct.C; i += kWave) smem[oP + i] = m.fpose[12 * ct.frame[i / 12] + i % 12];
        for (int i = t; i < ct.C; i += kWave) smem[oL + i] = (double)m.flink[ct.frame[i]];
        wave_sync();
        m.jaxis = smem + oA;
        m.jrot = smem + oR;
        m.com = smem + oC;
        m.inertia = smem + oI;
        m.mass = smem + oM;
        m.cpose = smem + oP;
        m.clink = smem + oL;
        if (imp.kp) {
            imp.kp = smem + oKp;
            imp.kd = smem + oKd;
        }
    }
    constexpr int per = kWave / HW;   // systems per wavefront
    const Topo T = build_topo<HW>(m, S);
    double* loc = S.st();   // bv 6 | jv n | bp 3 | bR 9 | jp n | dR 9
    double* dR = loc + 18 + 2 * n;
    const int64_t i0 = (int64_t)blockIdx.x * per + H.half;
    // a system past the end of an odd batch is computed (as the last system's copy, beside its
    // partner) and written nowhere
    const bool active = i0 < batch;   // see fbd_dynamics_kernel
    const int64_t q = active ? i0 : batch - 1;
    for (int i = lane; i < 18 + 2 * n; i += HW) {
        double v;
        if (i < 6) v = st.base_vel[6 * q + i];
        else if (i < 6 + n) v = st.joint_vel[(int64_t)n * q + (i - 6)];
        else if (i < 9 + n) v = st.base_pos[3 * q + (i - 6 - n)];
        else if (i < 18 + n) v = st.base_rot[9 * q + (i - 9 - n)];
        else v = st.joint_pos[(int64_t)n * q + (i - 18 - n)];
        loc[i] = v;
    }
    if constexpr (kCS) {   // this system's constants of the Euler loop, once (BLF_FBD_CSTAGE)
        const int C = ct.C;
        for (int i = lane; i < 29 * C; i += HW) {
            double v;
            if (i < C) v = (double)m.flink[ct.frame[i]];
            else if (i < 13 * C) v = m.fpose[12 * ct.frame[(i - C) / 12] + (i - C) % 12];
            else if (i < 25 * C) v = ct.null_pose[(q * C) * 12 + (i - 13 * C)];
            else v = ct.params[i - 25 * C];
            S.cst()[i] = v;
        }
        if (imp.kp)
            for (int j = lane; j < n; j += HW) {
                S.imp()[j] = imp.kp[j];
                S.imp()[n + j] = imp.kd[j];
                S.imp()[2 * n + j] = imp.qref[(int64_t)n * q + j];
            }
    }
    wave_sync();
    bool ok = true;
    const double* tq = tau + (int64_t)n * q;
    for (int32_t step = 0; step < nsteps; ++step) {
        const double h = step + 1 < nsteps ? dT : dT_last;
        if (imp.kp) {   // the control input of this step from its start state
            for (int j = lane; j < n; j += HW) {
                if constexpr (kCS)
                    S.tq()[j] = S.imp()[j] * (S.imp()[2 * n + j] - loc[18 + n + j]) - S.imp()[n + j] * loc[6 + j];
                else
                    S.tq()[j] = imp.kp[j] * (imp.qref[(int64_t)n * q + j] - loc[18 + n + j]) - imp.kd[j] * loc[6 + j];
            }
            wave_sync();
            tq = S.tq();
        }
        ok = fbd_eval<NVMAX, HW, PRI, BLF_FBD_FOLD, kLM, kCS, ABA>(m, S, loc, loc + 6, loc + 6 + n, loc + 9 + n, loc + 18 + n,
                                 tq, ct, q, reg, T) && ok;
        if (lane == 0) fbk_rot_rate(m.rho, loc + 9 + n, loc + 3, dR);
        wave_sync();
        // every element moves by its derivative at the start of the step (ForwardEuler.tpp:37-45):
        // positions first (they read the old velocities), then the velocities
        for (int i = lane; i < 12 + n; i += HW) {
            // base position (3), base rotation (9), joint positions (n)
            if (i < 3) loc[6 + n + i] = loc[6 + n + i] + loc[i] * h;
            else if (i < 12) loc[6 + n + i] = loc[6 + n + i] + dR[i - 3] * h;
            else loc[18 + n + (i - 12)] = loc[18 + n + (i - 12)] + loc[6 + (i - 12)] * h;
        }
        wave_sync();
        for (int i = lane; i < NV; i += HW) loc[i] = loc[i] + S.rhs()[i] * h;
        wave_sync();
    }
    if (active) {
        const double nan = __builtin_nan("");
        for (int i = lane; i < 18 + 2 * n; i += HW) {
            const double v = ok ? loc[i] : nan;
            if (i < 6) st.base_vel[6 * q + i] = v;
            else if (i < 6 + n) st.joint_vel[(int64_t)n * q + (i - 6)] = v;
            else if (i < 9 + n) st.base_pos[3 * q + (i - 6 - n)] = v;
            else if (i < 18 + n) st.base_rot[9 * q + (i - 9 - n)] = v;
            else st.joint_pos[(int64_t)n * q + (i - 18 - n)] = v;
        }
    }
}

// The closed loop's state -> plan map: the centre of mass, its velocity
// and the DCM of every system,
//   c = sum_l m_l (p_l + R_l com_l) / m,   cdot = sum_l m_l (v_l + w_l x R_l com_l) / m,
//   xi = c_xy + cdot_xy / omega_0
// (the LIP's divergent component with the plan's first-knot omega).  One wavefront per system:
// the forward kinematics of fbd_eval, then lane per link and one wave sum per quantity.
template <bool PRI>
__global__ __launch_bounds__(64) void fb_dcm_kernel(Model m, blf_fb_state st, const double* __restrict__ omega0,
                                                    int64_t ostride, double* __restrict__ com,
                                                    double* __restrict__ xi)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int n = m.n, L = n + 1;
    const Smem S(smem, n, 0, true);   // kinematics only: the compact (articulated-body) layout
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x;
    double* loc = S.st();   // bv 6 | jv n | bp 3 | bR 9 | jp n
    for (int i = lane; i < 18 + 2 * n; i += kWave) {
        double v;
        if (i < 6) v = st.base_vel[6 * q + i];
        else if (i < 6 + n) v = st.joint_vel[(int64_t)n * q + (i - 6)];
        else if (i < 9 + n) v = st.base_pos[3 * q + (i - 6 - n)];
        else if (i < 18 + n) v = st.base_rot[9 * q + (i - 9 - n)];
        else v = st.joint_pos[(int64_t)n * q + (i - 18 - n)];
        loc[i] = v;
    }
    wave_sync();
    const Topo T = build_topo<kWave>(m, S);
    fbd_kinematics<kWave, PRI>(m, S, loc, loc + 6, loc + 6 + n, loc + 9 + n, loc + 18 + n, T);
    wave_sync();
    double a[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};   // m c (3), m cdot (3), m
    if (lane < L) {
        const double* k = S.link() + S.lrec * lane;
        const double* R = k + kR;
        const double* cl = m.com + 3 * lane;
        double rc[3], t[3];
        for (int i = 0; i < 3; ++i) rc[i] = (R[3 * i] * cl[0] + R[3 * i + 1] * cl[1]) + R[3 * i + 2] * cl[2];
        cross3(k + kW, rc, t);
        const double ms = m.mass[lane];
        for (int i = 0; i < 3; ++i) {
            a[i] = ms * (k[kP + i] + rc[i]);
            a[3 + i] = ms * (k[kV + i] + t[i]);
        }
        a[6] = ms;
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) a[i] = wave_sum(a[i]);
    if (lane == 0) {
        double o[6];
        for (int i = 0; i < 6; ++i) o[i] = a[i] / a[6];
        for (int i = 0; i < 6; ++i) com[6 * q + i] = o[i];
        if (xi) {
            const double w0 = omega0[q * ostride];
            xi[2 * q] = o[0] + o[3] / w0;
            xi[2 * q + 1] = o[1] + o[4] / w0;
        }
    }
}

// The world transform and mixed twist of K frames of every system (blf_fb_frame_state): the state
// a caller hands a ContactModel it evaluates itself (BLF_CONTACT_WRENCH).  One wavefront per
// system: the forward kinematics of fbd_eval, then lane per frame with fbd_eval's own frame_state.
template <bool PRI>
__global__ __launch_bounds__(64) void fb_frame_state_kernel(Model m, blf_fb_state st, int K,
                                                            const int32_t* __restrict__ frames,
                                                            double* __restrict__ pose,
                                                            double* __restrict__ twist)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int n = m.n;
    const Smem S(smem, n, 0, true);   // kinematics only: the compact (articulated-body) layout
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x;
    double* loc = S.st();   // bv 6 | jv n | bp 3 | bR 9 | jp n
    for (int i = lane; i < 18 + 2 * n; i += kWave) {
        double v;
        if (i < 6) v = st.base_vel[6 * q + i];
        else if (i < 6 + n) v = st.joint_vel[(int64_t)n * q + (i - 6)];
        else if (i < 9 + n) v = st.base_pos[3 * q + (i - 6 - n)];
        else if (i < 18 + n) v = st.base_rot[9 * q + (i - 9 - n)];
        else v = st.joint_pos[(int64_t)n * q + (i - 18 - n)];
        loc[i] = v;
    }
    wave_sync();
    const Topo T = build_topo<kWave>(m, S);
    fbd_kinematics<kWave, PRI>(m, S, loc, loc + 6, loc + 6 + n, loc + 9 + n, loc + 18 + n, T);
    wave_sync();
    for (int c = lane; c < K; c += kWave) {
        const int f = frames[c];
        double p[12], tw[6];
        if (f >= 0 && f < m.F) {
            frame_state(S.link() + S.lrec * m.flink[f], m.fpose + 12 * f, p, tw);
        } else {   // a frame index outside [0, nframes): NaN, never an out-of-bounds read
            for (int a = 0; a < 12; ++a) p[a] = __builtin_nan("");
            for (int a = 0; a < 6; ++a) tw[a] = __builtin_nan("");
        }
        if (pose)
            for (int a = 0; a < 12; ++a) pose[(q * K + c) * 12 + a] = p[a];
        if (twist)
            for (int a = 0; a < 6; ++a) twist[(q * K + c) * 6 + a] = tw[a];
    }
}

// The closed loop's plan -> robot map: the joint references held over one
// control period,
//   q_ref_j = q_nom_j + lean_j0 (r0_x - c_x) + lean_j1 (r0_y - c_y)
// with r0 the plan's first VRP and c the centre of mass; the joint impedance of
// fbd_euler_kernel tracks them.  Element per (system, joint).
__global__ __launch_bounds__(256) void posture_reference_kernel(int n, const double* __restrict__ qnom,
                                                                const double* __restrict__ lean,
                                                                const double* __restrict__ com,
                                                                const double* __restrict__ vrp,
                                                                int64_t vstride, int64_t total,
                                                                double* __restrict__ qref)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int64_t q = e / n;
    const int j = (int)(e - q * n);
    const double ex = vrp[q * vstride] - com[6 * q];
    const double ey = vrp[q * vstride + 1] - com[6 * q + 1];
    qref[e] = (qnom[j] + lean[2 * j] * ex) + lean[2 * j + 1] * ey;
}

Model to_model(const blf_fb_model* md)
{
    Model m;
    m.n = md->ndof;
    m.F = md->nframes;
    m.parent = md->parent;
    m.jorig = md->joint_origin;
    m.jrot = md->joint_rot;
    m.jaxis = md->joint_axis;
    m.mass = md->link_mass;
    m.com = md->link_com;
    m.inertia = md->link_inertia;
    m.flink = md->frame_link;
    m.fpose = md->frame_pose;
    m.cpose = nullptr;
    m.clink = nullptr;
    m.g0 = md->gravity[0];
    m.g1 = md->gravity[1];
    m.g2 = md->gravity[2];
    m.rho = md->rho;
    m.jtype = md->joint_type;
    return m;
}

Contacts to_contacts(const blf_fb_contacts* c)
{
    Contacts o;
    o.C = c ? c->ncontacts : 0;
    o.frame = c ? c->frame : nullptr;
    o.params = c ? c->params : nullptr;
    o.null_pose = c ? c->null_pose : nullptr;
    o.law = c ? c->law : nullptr;
    o.wrench = c ? c->wrench : nullptr;
    return o;
}

}  // namespace

size_t fbd_lds_bytes(int n, int C, bool aba) { return sizeof(double) * Smem(nullptr, n, C, aba).total; }

// The articulated-body solve (fbd_aba) unless the model carries a mass-matrix regularisation,
// which needs M itself; BLF_FBD_ABA=0 keeps the factorization for every model (A/B only).
static bool use_aba(const double* reg)
{
    static const bool on = [] {
        const char* e = getenv("BLF_FBD_ABA");
        return !(e && e[0] == '0');
    }();
    return on && reg == nullptr;
}

blf_status launch_fbd_dynamics(const blf_fb_model* md, const blf_fb_state* st, const double* tau,
                               const blf_fb_contacts* ct, const double* reg, int64_t batch,
                               const blf_fb_state* out, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const Contacts c = to_contacts(ct);
    const bool pri = md->joint_type != nullptr, aba = use_aba(reg);
    const size_t lds = fbd_lds_bytes(md->ndof, c.C, aba);
#define FBD_DYN(NV, HW) (pri ? (aba ? fbd_dynamics_kernel<NV, HW, true, true> : fbd_dynamics_kernel<NV, HW, true, false>) \
                             : (aba ? fbd_dynamics_kernel<NV, HW, false, true> : fbd_dynamics_kernel<NV, HW, false, false>))
    if (md->ndof + 6 <= 32)   // two systems per wavefront
        hipLaunchKernelGGL(FBD_DYN(32, 32), dim3((unsigned)ceil_div(batch, 2)), dim3(kWave), 2 * lds, s,
                           to_model(md), *st, tau, c, reg, *out, batch);
    else
        hipLaunchKernelGGL(FBD_DYN(BLF_FBD_MAX_DOFS + 6, kWave), dim3((unsigned)batch), dim3(kWave), lds, s,
                           to_model(md), *st, tau, c, reg, *out, batch);
#undef FBD_DYN
    return check_hip(hipGetLastError(), "fbd_dynamics_kernel launch");
}

blf_status launch_fbd_euler(const blf_fb_model* md, const blf_fb_state* st, const double* tau,
                            const blf_fb_contacts* ct, const double* reg, int64_t batch,
                            int32_t nsteps, double dT, double dT_last, hipStream_t s,
                            const blf_joint_impedance* impedance)
{
    if (batch == 0) return BLF_OK;
    const size_t mb32 = BLF_FBD_LDSMODEL ? sizeof(double) * fbd_model_block<32>() : 0;
    const Contacts c = to_contacts(ct);
    Impedance imp{nullptr, nullptr, nullptr};
    if (impedance) imp = Impedance{impedance->kp, impedance->kd, impedance->q_ref};
    const bool pri = md->joint_type != nullptr, aba = use_aba(reg);
    const size_t lds = fbd_lds_bytes(md->ndof, c.C, aba);
#define FBD_EUL(NV, HW) (pri ? (aba ? fbd_euler_kernel<NV, HW, true, true> : fbd_euler_kernel<NV, HW, true, false>) \
                             : (aba ? fbd_euler_kernel<NV, HW, false, true> : fbd_euler_kernel<NV, HW, false, false>))
    if (md->ndof + 6 <= 32)   // two systems per wavefront
        hipLaunchKernelGGL(FBD_EUL(32, 32), dim3((unsigned)ceil_div(batch, 2)), dim3(kWave), 2 * lds + mb32, s,
                           to_model(md), *st, tau, c, reg, nsteps, dT, dT_last, imp, batch);
    else
        hipLaunchKernelGGL(FBD_EUL(BLF_FBD_MAX_DOFS + 6, kWave), dim3((unsigned)batch), dim3(kWave), lds, s,
                           to_model(md), *st, tau, c, reg, nsteps, dT, dT_last, imp, batch);
#undef FBD_EUL
    return check_hip(hipGetLastError(), "fbd_euler_kernel launch");
}

blf_status launch_fb_dcm(const blf_fb_model* md, const blf_fb_state* st, const double* omega0,
                         int64_t ostride, int64_t batch, double* com, double* xi, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const size_t lds = fbd_lds_bytes(md->ndof, 0, true);
    hipLaunchKernelGGL((md->joint_type ? fb_dcm_kernel<true> : fb_dcm_kernel<false>), dim3((unsigned)batch),
                       dim3(kWave), lds, s, to_model(md), *st,
                       omega0, ostride, com, xi);
    return check_hip(hipGetLastError(), "fb_dcm_kernel launch");
}

blf_status launch_fb_frame_state(const blf_fb_model* md, const blf_fb_state* st, int32_t K,
                                 const int32_t* frames, int64_t batch, double* pose, double* twist,
                                 hipStream_t s)
{
    if (batch == 0 || K == 0) return BLF_OK;
    const size_t lds = fbd_lds_bytes(md->ndof, 0, true);
    hipLaunchKernelGGL((md->joint_type ? fb_frame_state_kernel<true> : fb_frame_state_kernel<false>),
                       dim3((unsigned)batch), dim3(kWave), lds, s, to_model(md), *st, (int)K, frames,
                       pose, twist);
    return check_hip(hipGetLastError(), "fb_frame_state_kernel launch");
}

blf_status launch_posture_reference(const blf_posture_law* law, const double* com, const double* vrp,
                                    int64_t vstride, int64_t batch, double* qref, hipStream_t s)
{
    const int64_t total = batch * law->ndof;
    if (total == 0) return BLF_OK;
    hipLaunchKernelGGL(posture_reference_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, s,
                       law->ndof, law->q_nominal, law->lean, com, vrp, vstride, total, qref);
    return check_hip(hipGetLastError(), "posture_reference_kernel launch");
}

}  // namespace blf
