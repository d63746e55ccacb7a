// mjh_step.hip — batched mj_step / mj_forward for gfx950 (MI355X).
//
// One workgroup per world. Every per-world intermediate (poses, com inertias,
// mass matrix and its factor, contacts, constraint Jacobian, solver state)
// lives in LDS for the whole step; HBM is touched once to read the state and
// once to write the outputs (world-outermost arrays, see mjh_fields.h).
// Lanes are spread over the world's inner dimensions: bodies (kinematic chains
// are walked per lane, no per-level barriers), dofs, geom pairs, constraint
// rows and lower-triangle matrix entries. Per-world reductions are wave
// butterflies (__shfl_xor) + an LDS combine across waves; compaction of
// contacts / constraint rows uses a block exclusive scan, so contact and row
// order is deterministic (pair-table order, as MuJoCo's collision driver).
//
// Pipeline (MuJoCo's mj_step; reference call sites sim.py:138-147,186-199):
//   kinematics -> com_pos -> crb -> LDL^T(M) -> collision -> make_constraint
//   -> com_vel/rne -> passive/actuation -> qacc_smooth -> Newton solve
//   -> post-constraint acc -> sensors -> implicitfast / Euler integration.
// Solver options follow mjlab's MujocoCfg (sim.py:42-76): Newton, pyramidal
// cones, exact line search, tolerance scaled by meaninertia.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <string>
#include <type_traits>

#include "../../include/mjh_abi.h"
#include "mjh_convex.h"
#include "mjh_math.h"
#include "mjh_rng.h"

using namespace mjh;

namespace {

// Per-world LDS layout, offsets in 4-byte words from the world's base.
struct Layout {
  int qpos, qvel, qacc, qacc_smooth, qfrc_smooth, qfrc_bias, qfrc_con, qfrc_passive, qfrc_act;
  int grad, search, Ma, Mv, tmp, tmp2;
  int xpos, xquat, xmat, xipos, ximat, subtree_com, cinert, crb, cvel, cacc, cfrc;
  int xanchor, xaxis, cdof, cdof_dot;
  int cgpos, cgmat, sxpos, sxmat;
  int M, L, ldm;
  int act_force;
  int con_pos, con_frame, con_dist, con_fric, con_solref, con_solimp, con_imargin, con_dim, con_geom, con_efcadr;
  int J, ldj, efc_D, efc_R, efc_aref, efc_jaref, efc_jv, efc_force, efc_fl, efc_pos, efc_type, efc_id, efc_mask;
  int efc_h, arow, ash;
  int sidx;  // contact sensor: kept matches (contact index, ~index if flipped)
  int cg_g, cg_mg;  // CG solver: the previous iteration's gradient and M^-1 gradient
  int pgs_ar, pgs_mj;  // PGS solver (global scratch): AR = J M^-1 J' + R (rcap x rcap), rows M^-1 J_r'
  int red, ints;
  int total, gtotal;  // per-world words: LDS, global scratch
  int ncap, rcap;
  // one-world workgroups: the LDS holds the row arrays for lcap rows; a world
  // with more (up to rcap = njmax) keeps them at these global-scratch offsets
  int lcap;
  int g_efc_D, g_efc_R, g_efc_aref, g_efc_jaref, g_efc_jv, g_efc_force, g_efc_fl, g_efc_type, g_efc_h, g_arow, g_ash;
  // split step (MODE 1 position kernel -> MODE 2 velocity/solver kernel): the
  // position kernel's outputs that the full kernel keeps in LDS go through a
  // per-world global handoff region, plus the reuse snapshot
  int h_L, h_type, h_fl, h_D, h_R, h_aref, h_b, h_jv, h_ints, h_snap;
  int pred, pints, ptotal;  // the position kernel's per-world LDS (qpos + reductions)
};

enum { I_NCON = 0, I_NEFC, I_FLAGS, I_NITER, I_MISC, I_COUNT = 8 };
constexpr int kSolverPGS = 0, kSolverCG = 1;  // mjtSolver: mjSOL_PGS 0, mjSOL_CG 1, mjSOL_NEWTON 2

// Where each per-world array lives: LDS (fast, but it bounds how many worlds
// share a CU) or the per-world global scratch (L1/L2-resident; coalesced since
// a world's scratch is one contiguous span). The solver's hot set — J, the row
// state and the nv-vectors — stays in LDS; poses, inertias, contacts and the
// mass matrix go to global scratch so more worlds (waves) fit per CU.
// Inlining the solver helpers trades call overhead (callee-saved VGPR spills,
// flat addressing of LDS through generic pointers) for register pressure.
#ifndef MJH_SOLVER_INLINE
#define MJH_SOLVER_INLINE
#endif
#ifndef MJH_COLL_INLINE
#define MJH_COLL_INLINE
#endif
#ifndef MJH_PRESET
#define MJH_PRESET 5
#endif
// the Newton direction after a Hessian rebuild: factor with the forward
// substitution fused into its sweep (1) or factor, then solve (0)
#ifndef MJH_FUSED_FWD
#define MJH_FUSED_FWD 0
#endif
// collision pairs read from per-pair records the pack launch writes (1) or
// through the pair and geom arrays (0): see make_imgoff
#ifndef MJH_PAIR_REC
#define MJH_PAIR_REC 1
#endif
// sensor-phase variants (contact sensors: metadata preload, match test from
// registers, LDS-only fences): A/B switches, see the sensor phase. Measured
// (profiles/r06f_sensor_ab.log, G1 4096 kernel_bench, two passes): preload packed
// 0.495 / 0.492 vs 0.498 / 0.500 ms (adopted); LDS-only fences no change; the
// match test from registers (6 more live registers) 0.514 ms; unpacked preload
// (10 registers) 0.527 ms (profiles/r06e) — the allocator moved spills into the solver
#ifndef MJH_SENS_PRELOAD
#define MJH_SENS_PRELOAD 2
#endif
#ifndef MJH_SENS_OMREG
#define MJH_SENS_OMREG 0
#endif
#ifndef MJH_SENS_LSYNC
#define MJH_SENS_LSYNC 0
#endif
// cacc's chain sum over lane-formed per-dof terms (6 readlanes per dof instead of
// 14). Measured (profiles/r06p_cacc_ab_kb.log): Go1 0.415 -> 0.409 ms per launch, G1 flat
#ifndef MJH_CACC_W
#define MJH_CACC_W 1
#endif
// every contact sensor's matches computed in one pass before the first sensor
// output is stored (ballots per sensor in the solver's dead ash array): the match
// test's dependent image loads run once, not once per contact sensor behind the
// previous sensors' stores. Measured (profiles/r06o_prematch_ab_kb.log): G1 0.471 ->
// 0.478 ms per launch (VGPR spills 119 -> 192), Go1 flat: off
#ifndef MJH_SENS_PREMATCH
#define MJH_SENS_PREMATCH 0
#endif
#define MJH_REGIONS(X)                                                                              \
  X(qpos, 0) X(qvel, 0) X(qacc, 0) X(qacc_smooth, 0) X(qfrc_smooth, 0) X(qfrc_bias, 1) X(qfrc_con, 0)  \
  X(qfrc_passive, 1) X(qfrc_act, 1) X(grad, 0) X(search, 0) X(Ma, 0) X(Mv, 0) X(tmp, 0) X(tmp2, 0)    \
  X(xpos, 1) X(xquat, 1) X(xmat, 1) X(xipos, 1) X(ximat, 1) X(subtree_com, 1) X(cinert, 0) X(crb, 0)  \
  X(cvel, 0) X(cacc, 1) X(cfrc, 0) X(xanchor, 1) X(xaxis, 1) X(cdof, 0) X(cdof_dot, 0)               \
  X(cgpos, 1) X(cgmat, 1) X(sxpos, 1) X(sxmat, 1) X(M, 1) X(L, 1) X(act_force, 1)                    \
  X(con_pos, 1) X(con_frame, 1) X(con_dist, 1) X(con_fric, 1) X(con_solref, 1) X(con_solimp, 1)       \
  X(con_imargin, 1) X(con_dim, 1) X(con_geom, 1) X(con_efcadr, 1)                                     \
  X(J, 0) X(efc_D, 0) X(efc_R, 0) X(efc_aref, 0) X(efc_jaref, 0) X(efc_jv, 0) X(efc_force, 0)        \
  X(efc_fl, 0) X(efc_pos, 1) X(efc_type, 0) X(efc_id, 1) X(efc_mask, 1) X(efc_h, 0) X(arow, 0)       \
  X(ash, 0) X(sidx, 1) X(cg_g, 1) X(cg_mg, 1)
struct Rg {
#if MJH_PRESET == 0
#define X_RG(name, r) static constexpr bool name = false;
#elif MJH_PRESET == 2
#define X_RG(name, r) static constexpr bool name = true;
#elif MJH_PRESET == 4
#define X_RG(name, r) static constexpr bool name = (r) != 0 || (#name[0] == 'J' && #name[1] == 0) || \
    (#name[0] == 'c' && (#name[1] == 'i' || #name[1] == 'r' || #name[1] == 'v' || #name[1] == 'f' || #name[1] == 'd'));
#elif MJH_PRESET == 5
// like 4 (body arrays global) but the mass-matrix / Hessian factor L in LDS
#define X_RG(name, r) static constexpr bool name = ((r) != 0 || (#name[0] == 'J' && #name[1] == 0) || \
    (#name[0] == 'c' && (#name[1] == 'i' || #name[1] == 'r' || #name[1] == 'v' || #name[1] == 'f' || #name[1] == 'd'))) && \
    !(#name[0] == 'L' && #name[1] == 0);
#elif MJH_PRESET == 6
// like 5, and the constraint-row arrays in global scratch as well: ~7 KB of LDS
// per world (nv-vectors + the factor), so 16 worlds share a CU and rcap = njmax
#define X_RG(name, r) static constexpr bool name = ((r) != 0 || (#name[0] == 'J' && #name[1] == 0) || \
    (#name[0] == 'c' && (#name[1] == 'i' || #name[1] == 'r' || #name[1] == 'v' || #name[1] == 'f' || #name[1] == 'd')) || \
    (#name[0] == 'e' && #name[1] == 'f' && #name[2] == 'c') || (#name[0] == 'a' && (#name[1] == 'r' || #name[1] == 's'))) && \
    !(#name[0] == 'L' && #name[1] == 0);
#elif MJH_PRESET == 7
// like 4 (body arrays, J and the factor L in global scratch), and the
// constraint rows' colder arrays as well (R, frictionloss, aref, the active-set
// lists): ~6 words of LDS per row, so 300 rows fit 16 worlds per CU
#define X_RG(name, r) static constexpr bool name = (r) != 0 || (#name[0] == 'J' && #name[1] == 0) || \
    (#name[0] == 'L' && #name[1] == 0) || \
    (#name[0] == 'c' && (#name[1] == 'i' || #name[1] == 'r' || #name[1] == 'v' || #name[1] == 'f' || #name[1] == 'd')) || \
    (#name[0] == 'e' && #name[1] == 'f' && #name[2] == 'c' && #name[3] == '_' && \
     ((#name[4] == 'R' && #name[5] == 0) || (#name[4] == 'f' && #name[5] == 'l') || (#name[4] == 'a' && #name[5] == 'r'))) || \
    (#name[0] == 'a' && (#name[1] == 'r' || #name[1] == 's'));
#elif MJH_PRESET == 3
#define X_RG(name, r) static constexpr bool name = (r) != 0 || (#name[0] == 'J' && #name[1] == 0);
#else
#define X_RG(name, r) static constexpr bool name = (r) != 0;
#endif
  MJH_REGIONS(X_RG)
#undef X_RG
};
// Position reuse and the split step read the position stage's results from a
// later launch. The handoff area restores the factor of M, the rows' position
// parameters and the counters; every other array the stage writes and the
// velocity/solver/sensor stages read must sit in global scratch, where the last
// launch left it (an LDS copy belongs to whatever ran on that CU since).
constexpr bool kPositionStageGlobal =
    Rg::xpos && Rg::xquat && Rg::xmat && Rg::xipos && Rg::ximat && Rg::subtree_com && Rg::cinert && Rg::crb &&
    Rg::cdof && Rg::xanchor && Rg::xaxis && Rg::cgpos && Rg::cgmat && Rg::sxpos && Rg::sxmat && Rg::M && Rg::J &&
    Rg::con_pos && Rg::con_frame && Rg::con_dist && Rg::con_fric && Rg::con_solref && Rg::con_solimp &&
    Rg::con_imargin && Rg::con_dim && Rg::con_geom && Rg::con_efcadr && Rg::efc_pos && Rg::efc_id && Rg::efc_mask &&
    Rg::sidx;
#define SP(name) ((Rg::name ? G : S) + Lo.name)
#define SPI(name) reinterpret_cast<int*>((Rg::name ? G : S) + Lo.name)

thread_local std::string g_err;
thread_local bool g_keep_image = false;  // mjh_step_keep_image: no pack launch before this step
bool g_disable_spec = false;  // mjh_set_specialization(0): always the generic instance
bool g_auto_order = false;    // mjh_set_world_ordering(1): order the worlds in the pack launch
bool g_pos_reuse = kPositionStageGlobal;  // mjh_set_position_reuse: reuse the position stage of unchanged worlds
int g_lds_row_cap = 0;  // mjh_set_lds_row_cap: test cap on the LDS-resident constraint rows (0: none)
#ifndef MJH_SPLIT
#define MJH_SPLIT 0
#endif
static_assert(MJH_SPLIT == 0 || kPositionStageGlobal,
              "MJH_SPLIT hands the position stage over in global scratch: this MJH_PRESET keeps part of it in LDS");
#ifndef MJH_PWPB
#define MJH_PWPB 8
#endif

#ifdef MJH_PROFILE
#ifndef MJH_LSDBG_IT
#define MJH_LSDBG_IT 0
#endif
__device__ unsigned long long* g_prof;
__device__ float* g_lsdbg;  // (nworld, 32) candidate costs of the parallel line search (diagnostics)
#define PROF(k)                                                           \
  do {                                                                    \
    wsync();                                                              \
    if (tid == 0 && g_prof) g_prof[(long long)w * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define PROF_ACC(k, t0)                                                   \
  do {                                                                    \
    wsync();                                                              \
    if (tid == 0 && g_prof) g_prof[(long long)w * 32 + (k)] += __builtin_amdgcn_s_memtime() - (t0); \
  } while (0)
#define PROF_NOW() __builtin_amdgcn_s_memtime()
#else
#define PROF(k) do {} while (0)
#define PROF_ACC(k, t0) do {} while (0)
#define PROF_NOW() 0ull
#endif

// Wave-level synchronisation: one world = one wave. DS instructions of a wave
// execute in issue order, so lanes exchanging data through LDS only need the
// compiler not to move LDS accesses across this point (memory clobber) and the
// outstanding LDS ops drained; no s_barrier, so waves of a workgroup that run
// different worlds never wait for each other.
// Per-world arrays in global scratch are exchanged the same way: all waves of
// a workgroup share the CU's L1, so draining vmcnt makes a lane's stores
// visible to the wave's other lanes (workgroup scope, non-tgsplit).
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); }
// LDS-only fence (and a compiler barrier): a wave's LDS operations execute in
// issue order, so this orders its LDS traffic without waiting for its
// outstanding global stores as wsync does (vmcnt counts stores on gfx9)
__device__ __forceinline__ void lsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Bounds-check builds (-DMJH_BOUNDS=1, tools/bounds_check.py): an index outside its
// array's capacity skips the access and sets MJH_FLAG_BOUNDS in the world's flags
// (an LDS atomic on the world's counters, no trap); other builds compile to true.
#ifndef MJH_BOUNDS
#define MJH_BOUNDS 0
#endif
#if MJH_BOUNDS
#define MJH_BOK(idx, cap) \
  (((unsigned)(idx) < (unsigned)(cap)) ? true : (atomicOr(&ints[I_FLAGS], MJH_FLAG_BOUNDS), false))
#else
#define MJH_BOK(idx, cap) true
#endif

// Word offsets of every model array inside the LDS model image, and of the
// per-world copies of expanded (domain-randomised) fields (-1: shared).
struct ImgOff {
#define X_IO(type, name, count) int name;
  MJH_MODEL_ARRAYS(X_IO)
  MJH_MODEL_WARRAYS(X_IO)
#undef X_IO
#define X_IOW(type, name, count) int w_##name;
  MJH_MODEL_WARRAYS(X_IOW)
#undef X_IOW
  int pair_rec;  // the collision pairs' records (pack_kernel; MJH_PAIR_REC)
  int img_words;
  int nfields;
};

#ifndef MJH_WPCU
#define MJH_WPCU 16  // resident worlds per CU (see MJH_MINWAVES)
#endif
// Worlds per workgroup by padded dof count. 21-36 dofs (G1): one-world
// workgroups; each wave retires on its own, the model image is read in place
// from global memory, and MJH_WPCU (16) of them share a CU — 4 waves per SIMD, so
// all 4,096 G1 worlds are resident at once (one round instead of two; G1 step
// launch 0.605 -> 0.505 ms, env bench 1.37M -> 1.57M env-steps/s,
// profiles/r04m_*). Up to 20 dofs (Go1): one workgroup of MJH_WPCU worlds per CU
// sharing an LDS copy of the image (Go1 8192 0.523 -> 0.501 ms; for G1 the
// smaller per-world LDS costs more than the image reads save,
// profiles/r04s_wg16_kb.log). 8-world workgroups sharing the image for larger
// models. MJH_WPB overrides it for A/B builds.
__host__ __device__ constexpr int wpb_of_nvp(int nvp) {
#ifdef MJH_WPB
  return (void)nvp, MJH_WPB;
#else
  return nvp <= 20 ? MJH_WPCU : (nvp <= 36 ? 1 : 8);
#endif
}
// the image lives in global memory for workgroups of fewer than 8 worlds
__host__ __device__ constexpr bool img_global(int wpb) { return wpb < 8; }
// one-world workgroups, and workgroups of a whole CU's MJH_WPCU worlds (one
// LDS copy of the image for all of them): per-world layouts sized for MJH_WPCU
// worlds per CU, with the packed factor, constraint rows beyond the LDS in
// global scratch (two tiers) and the world index in a scalar register
__host__ __device__ constexpr bool cu_worlds(int wpb) { return wpb == 1 || wpb == MJH_WPCU; }
template <bool G>
__device__ __forceinline__ const float* img_base(const float* g, const float* l) {
  if constexpr (G) return g; else return l;
}
#define IMGB imgb
#define IMG_I(name) (reinterpret_cast<const int*>(IMGB + Io.name))
#define IMG_F(name) (reinterpret_cast<const float*>(IMGB + Io.name))
#define IMG_L(name) (reinterpret_cast<const long long*>(IMGB + Io.name))
#define WFIELD(name) (m.name##_wstride ? (const float*)(m.name + W * m.name##_wstride) : (const float*)(IMGB + Io.name))

// ---- cross-lane exchange ------------------------------------------------------
// lane k's value to every lane (k wave-uniform): v_readlane_b32
__device__ __forceinline__ float rl(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
__device__ __forceinline__ unsigned long long rl64(unsigned long long v, int k) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, k), hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), k);
  return ((unsigned long long)hi << 32) | lo;
}
// lane src's value (src per lane): ds_bpermute; call with every lane active
__device__ __forceinline__ float shfl(float v, int src) { return __shfl(v, src, 64); }

// ---- wave primitives on DPP (no LDS round trips) -----------------------------
// dpp_ctrl: quad_perm 0x00-0xff, row_shr:n 0x110+n, row_mirror 0x140,
// row_half_mirror 0x141, row_bcast:15 0x142, row_bcast:31 0x143 (GFX9 DPP).
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf, bool BOUND_ZERO = true>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO));
}
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf, bool BOUND_ZERO = true>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO);
}

// sum over the 64 lanes, returned uniformly (lane 63 holds the total)
__device__ __forceinline__ float wave_sum(float v) {
  v += dppf<0xB1>(v);          // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);          // quad_perm [2,3,0,1]
  v += dppf<0x141>(v);         // row_half_mirror: 8-lane sums
  v += dppf<0x140>(v);         // row_mirror: 16-lane (row) sums
  v += dppf<0x142, 0xa>(v);    // row_bcast:15 into rows 1, 3
  v += dppf<0x143, 0xc>(v);    // row_bcast:31 into rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int a) {
  int x = a + dppi<0x111>(a) + dppi<0x112>(a) + dppi<0x113>(a);  // a[i-3..i] within the row
  x += dppi<0x114, 0xf, 0xe>(x);  // row_shr:4 into banks 1-3
  x += dppi<0x118, 0xf, 0xc>(x);  // row_shr:8 into banks 2-3
  x += dppi<0x142, 0xa, 0xf, false>(x);  // row_bcast:15 into rows 1, 3
  x += dppi<0x143, 0xc, 0xf, false>(x);  // row_bcast:31 into rows 2, 3
  return x;
}

// ---- block-level primitives -------------------------------------------------
template <int NT>
__device__ __forceinline__ float bsum(float v, float* red) {
  if constexpr (NT == 64) {
    return wave_sum(v);
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    wsync();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    wsync();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) s += red[i];
    return s;
  }
}

template <int NT>
__device__ __forceinline__ void bsum2(float& a, float& b, float* red) {
  if constexpr (NT == 64) {
    a = wave_sum(a);
    b = wave_sum(b);
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o, 64);
      b += __shfl_xor(b, o, 64);
    }
    wsync();
    if ((threadIdx.x & 63) == 0) {
      red[2 * (threadIdx.x >> 6)] = a;
      red[2 * (threadIdx.x >> 6) + 1] = b;
    }
    wsync();
    a = 0.f;
    b = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
      a += red[2 * i];
      b += red[2 * i + 1];
    }
  }
}

template <int NT>
__device__ __forceinline__ int bscan(int v, int* total, int* redi) {
  const int lane = threadIdx.x & 63;
  const int x = wave_incl_scan(v);
  if constexpr (NT == 64) {
    *total = __builtin_amdgcn_readlane(x, 63);
    return x - v;
  } else {
    const int wv = threadIdx.x >> 6;
    wsync();
    if (lane == 63) redi[wv] = x;
    wsync();
    int off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
      int t = redi[i];
      off += (i < wv) ? t : 0;
      tot += t;
    }
    *total = tot;
    return off + x - v;
  }
}

// index q of the "reversed" triangle -> (i, j) with i >= j, both in [n-m, n).
// Pairs with i, j >= n-m are exactly q < m(m+1)/2 (a prefix), which lets the
// factorisation walk a shrinking trailing block with one flat loop.
__device__ __forceinline__ void tri_rev(int q, int n, int& i, int& j) {
  int b = (int)((sqrtf(8.f * (float)q + 1.f) - 1.f) * 0.5f);
  while ((b + 1) * (b + 2) / 2 <= q) b++;
  while (b * (b + 1) / 2 > q) b--;
  int a = q - b * (b + 1) / 2;  // a <= b
  i = n - 1 - a;
  j = n - 1 - b;
}

// In-place LDL^T of the symmetric matrix in A (lower triangle used).
// On exit: strict lower = unit L, diagonal = D. One barrier per column: the
// scaling of column k-1 is deferred into pass k (disjoint addresses).
template <int NT>
__device__ void ldl_factor(float* A, int n, int ld) {
  const int tid = threadIdx.x & 63;
  float prev_inv = 0.f;
  for (int k = 0; k < n; k++) {
    wsync();
    float piv = A[k * ld + k];
    if (piv < MJH_MINVAL) piv = MJH_MINVAL;
    const float inv = 1.f / piv;
    const int mrem = n - 1 - k;  // trailing block size
    const int nitems = mrem * (mrem + 1) / 2;
    for (int q = tid; q < nitems; q += NT) {
      int i, j;
      tri_rev(q, n, i, j);
      A[i * ld + j] -= A[i * ld + k] * A[j * ld + k] * inv;
    }
    if (k > 0)
      for (int i = k + tid; i < n; i += NT) A[i * ld + (k - 1)] *= prev_inv;
    if (tid == 0) A[k * ld + k] = piv;
    prev_inv = inv;
  }
  wsync();
  (void)prev_inv;
}

// Left-looking (Crout) LDL^T for a single wave: lane i owns row i; column j is
// a dot product over the finished columns, pivots D[k] stay in registers and
// are broadcast with readlane. One wave barrier per column; all loads in the
// inner loop are independent (pipelined), unlike the right-looking update.
__device__ __forceinline__ float rdlane_f(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
template <int NT>
__device__ void ldl_factor_fast(float* A, int n, int ld) {
  if constexpr (NT != 64) {
    ldl_factor<NT>(A, n, ld);
  } else {
    const int lane = threadIdx.x & 63;
    float dreg = 0.f;
    const float* ri = A + lane * ld;
    for (int j = 0; j < n; j++) {
      wsync();
      float s = 0.f;
      if (lane >= j && lane < n) {
        const float* rj = A + j * ld;
        float acc0 = 0.f, acc1 = 0.f;
        int k = 0;
        for (; k + 4 <= j; k += 4) {
          const float4 a = *reinterpret_cast<const float4*>(ri + k);
          const float4 b = *reinterpret_cast<const float4*>(rj + k);
          acc0 += a.x * b.x * rdlane_f(dreg, k) + a.y * b.y * rdlane_f(dreg, k + 1);
          acc1 += a.z * b.z * rdlane_f(dreg, k + 2) + a.w * b.w * rdlane_f(dreg, k + 3);
        }
        for (; k < j; k++) acc0 += ri[k] * rj[k] * rdlane_f(dreg, k);
        s = ri[j] - (acc0 + acc1);
      }
      float dj = rdlane_f(s, j);
      if (dj < MJH_MINVAL) dj = MJH_MINVAL;
      if (lane == j) {
        dreg = dj;
        A[j * ld + j] = dj;
      } else if (lane > j && lane < n) {
        A[lane * ld + j] = s / dj;
      }
    }
    wsync();
  }
}

// Solve (L D L^T) x = x in place.
template <int NT>
__device__ void ldl_solve(const float* A, int n, int ld, float* x) {
  const int tid = threadIdx.x & 63;
  for (int k = 0; k < n; k++) {
    wsync();
    const float xk = x[k];
    for (int i = k + 1 + tid; i < n; i += NT) x[i] -= A[i * ld + k] * xk;
  }
  wsync();
  for (int i = tid; i < n; i += NT) x[i] /= A[i * ld + i];
  for (int k = n - 1; k > 0; k--) {
    wsync();
    const float xk = x[k];
    for (int i = tid; i < k; i += NT) x[i] -= A[k * ld + i] * xk;
  }
  wsync();
}

// Single-wave solve (n <= 64): x lives in one register per lane, the pivots of
// the forward/backward sweeps are broadcast with readlane (no LDS round trip,
// no barriers). Same arithmetic order as ldl_solve.
__device__ __forceinline__ float rdlane(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
template <int NT>
__device__ void ldl_solve_fast(const float* A, int n, int ld, float* x) {
  if constexpr (NT != 64) {
    ldl_solve<NT>(A, n, ld, x);
  } else {
    const int lane = threadIdx.x & 63;
    wsync();
    float xi = lane < n ? x[lane] : 0.f;
    const float* row = A + lane * ld;
    for (int k = 0; k < n - 1; k++) {
      const float xk = rdlane(xi, k);
      const float a = (lane > k && lane < n) ? row[k] : 0.f;
      xi -= a * xk;
    }
    if (lane < n) xi /= row[lane];
    for (int k = n - 1; k > 0; k--) {
      const float xk = rdlane(xi, k);
      const float a = lane < k ? A[k * ld + lane] : 0.f;
      xi -= a * xk;
    }
    if (lane < n) x[lane] = xi;
    wsync();
  }
}

// The factor L (and the Hessian it is factored from, and the mass matrix's
// staging rows) lives as packed lower-triangular rows: row i holds entries
// 0..i padded to a multiple of 4, 16-byte aligned. NVP rows take lrow(NVP)
// words (G1, NVP 36: 720 instead of 35 x 36 = 1,260), so more constraint rows
// fit the LDS. Entries right of the diagonal inside a row's padding are scratch.
// Packed for one-world workgroups (PK), whose LDS budget is tight; 8-world
// workgroups keep full rows of stride ld.
__host__ __device__ constexpr int lrow(int i) { return 4 * ((i >> 2) + 1) * (2 * (i >> 2) + (i & 3)); }
__host__ __device__ constexpr int llen(int i) { return ((i >> 2) + 1) << 2; }
static_assert(lrow(0) == 0 && lrow(1) == 4 && lrow(4) == 16 && lrow(5) == 24 && lrow(36) == 720, "packed rows");
template <bool PK> __device__ __forceinline__ int lofs(int i, int ld) { return PK ? lrow(i) : i * ld; }
template <bool PK> __device__ __forceinline__ int lspan(int i, int ld) { return PK ? llen(i) : ld; }
__host__ __device__ constexpr bool pack_l(int wpb) { return cu_worlds(wpb); }

// k-steps of J loads in flight in the Hessian, by padded dof count. Measured
// (profiles/r04pf_hess_pf_kb.log): G1 (36 dofs) flat across 2/4/6/8; Go1
// (20 dofs, ~14 rows: 6 covers all of them) 0.502 -> 0.457 ms per launch
#ifndef MJH_HESS_PF
#define MJH_HESS_PF(nvp) ((nvp) <= 20 ? 6 : 4)
#endif
// rows of J in flight per round of the solver's J^T f (a multiple of 4)
#ifndef MJH_JTF_B
#define MJH_JTF_B 16
#endif
// body / joint outputs computed in place in the data arrays (slab layout) instead of
// global scratch copied out at the end. Measured (profiles/r06y_out_direct_ab.log): G1
// 0.468 -> 0.454 ms, Go1 0.410 -> 0.405 ms per launch, env bench 1.707M -> 1.749M
#ifndef MJH_OUT_DIRECT
#define MJH_OUT_DIRECT 1
#endif
// contacts and sites computed in place in the data arrays too (A/B switch). Measured
// (gpurun_out r06z): G1 flat, Go1 0.405 -> 0.400 ms, 156 GPU tests green, but Go1's
// outputs are not bit-identical to the copy-out build (tools/lib_diff.py; G1's are): off
// until that difference is explained
#ifndef MJH_OUT_DIRECT2
#define MJH_OUT_DIRECT2 0
#endif
// kinematics by pointer jumping over the body tree (A/B switch). Measured
// (profiles/r06r_jtfpf_cdof_kinjump_ab_kb.log): G1 0.466 -> 0.459, Go1 0.409 -> 0.402 ms per
// launch, but the 40-step rollout parity test met a line-search choice beyond float32
// noise in one world (profiles/r06r_gputests_kinjump.log): off until that is explained
#ifndef MJH_KIN_JUMP
#define MJH_KIN_JUMP 0
#endif
// cdof rows built by dof lanes and kept in registers for the crb pass (A/B switch).
// Measured (same log): G1 0.466 -> 0.470, Go1 0.409 -> 0.407: off
#ifndef MJH_CDOF_LANE
#define MJH_CDOF_LANE 0
#endif
// J^T f's first round of loads issued ahead of the constraint-row pass (A/B switch).
// Measured (same log): flat on G1 and Go1: off
#ifndef MJH_JTF_PF
#define MJH_JTF_PF 0
#endif
// the Hessian's accumulators start from M's tiles with one 16-byte load per tile
// (M's symmetric rows, read transposed) instead of four scattered dword loads
#ifndef MJH_HESS_MROW
#define MJH_HESS_MROW 1
#endif
// H (lower triangle of Hout, packed rows) = M + sum_k ash[k]^2 J[arow[k]] J[arow[k]]^T over the
// nact compacted active rows, on the f32 matrix cores (v_mfma_f32_16x16x4_f32:
// exact fp32 FMA chains). Tiles of 16x16 on the lower block triangle; at most
// NB = NVP/16 (rounded up) tile rows. The accumulators start from M's lower
// triangle (its loads overlap the first J loads instead of trailing the loop).
template <int NT, int NVP, bool PK>
__device__ MJH_SOLVER_INLINE void hessian_mfma(const float* M, int ldm, const float* J, int ldj, const int* arow, const float* ash,
                             int nact, int n, float* Hout) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr int NB = (NVP + 15) / 16;
  constexpr int NTILE = NB * (NB + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int nb = (n + 15) >> 4;  // <= NB
  const int ci = lane & 15, kq = lane >> 4;
  v4f acc[NTILE];
  {
    int t = 0;
#pragma unroll
    for (int I = 0; I < NB; I++)
#pragma unroll
      for (int Jb = 0; Jb <= I; Jb++, t++) {
#if MJH_HESS_MROW
        // lane (ci, kq)'s entries (rows I*16+kq*4+q, column j = Jb*16+ci) are, M
        // being stored as whole symmetric rows, 4 consecutive entries of row j: one
        // 16-byte load. Entries never stored (right of the diagonal, rows or
        // columns >= n: padding zeros or row n-1's values) only pass through.
        const int j = Jb * 16 + ci, i0 = I * 16 + kq * 4;
        const float4 mv = i0 < n ? *reinterpret_cast<const float4*>(M + (j < n ? j : n - 1) * ldm + i0)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[t][0] = mv.x; acc[t][1] = mv.y; acc[t][2] = mv.z; acc[t][3] = mv.w;
#else
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int i = I * 16 + kq * 4 + q, j = Jb * 16 + ci;
          acc[t][q] = (i < n && j <= i) ? M[i * ldm + j] : 0.f;
        }
#endif
      }
  }
  // software pipeline: the next k-step's J values are loaded (J may live in
  // L2) while this step's MFMAs run
  auto load = [&](int k, float (&v)[NB]) {
    const int r = k < nact ? arow[k] : 0;
    const float sc = k < nact ? ash[k] : 0.f;
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int c = b * 16 + ci;
      v[b] = (b < nb && c < n) ? J[r * ldj + c] * sc : 0.f;
    }
  };
  // PF k-steps of J loads in flight (a ring unrolled by PF so every register
  // index is static); same k order as a plain loop, so the sums are unchanged
  constexpr int PF = MJH_HESS_PF(NVP);
  float v[PF][NB];
#pragma unroll
  for (int s = 0; s < PF; s++) load(4 * s + kq, v[s]);
  for (int k0 = 0; k0 < nact; k0 += 4 * PF) {
#pragma unroll
    for (int s = 0; s < PF; s++) {
      if (k0 + 4 * s < nact) {
        int t = 0;
#pragma unroll
        for (int I = 0; I < NB; I++)
#pragma unroll
          for (int Jb = 0; Jb <= I; Jb++, t++)
            if (I < nb) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[s][I], v[s][Jb], acc[t], 0, 0, 0);
      }
      if (k0 + 4 * (s + PF) < nact) load(k0 + 4 * (s + PF) + kq, v[s]);
    }
  }
  int t = 0;
#pragma unroll
  for (int I = 0; I < NB; I++)
#pragma unroll
    for (int Jb = 0; Jb <= I; Jb++, t++) {
      if (I >= nb) continue;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int i = I * 16 + kq * 4 + q, j = Jb * 16 + ci;
        if (i < n && j <= i) Hout[lofs<PK>(i, ldm) + j] = acc[t][q];
      }
    }
}

// Loads in flight per unrolled row dot: at most MJH_DOT_CHUNK entries of each
// operand are scheduled ahead (a scheduling barrier between chunks; 0: all of a
// row at once). Four waves per SIMD hide the latency the chunks expose, and the
// registers the whole-row form needs (two NVP-wide operands) do not fit 128.
#ifndef MJH_DOT_CHUNK
#define MJH_DOT_CHUNK 0
#endif
__device__ __forceinline__ void dot_chunk_barrier(int j) {
  if (MJH_DOT_CHUNK > 0 && j > 0 && (j % (MJH_DOT_CHUNK > 0 ? MJH_DOT_CHUNK : 1)) == 0) __builtin_amdgcn_sched_barrier(0);
}

// dot of an aligned row with an aligned vector, fully unrolled to the padded
// size NVP so all loads of a row are in flight at once (rows may live in L2);
// vector entries >= n are masked (padding may hold garbage)
template <int NVP>
__device__ __forceinline__ float rowdot_u(const float* r, const float* x, int n) {
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int j = 0; j < NVP; j += 4) {
    dot_chunk_barrier(j);
    const float4 a = *reinterpret_cast<const float4*>(r + j);
    float4 b = *reinterpret_cast<const float4*>(x + j);
    if (j + 4 > n) {
      b.x = j < n ? b.x : 0.f;
      b.y = j + 1 < n ? b.y : 0.f;
      b.z = j + 2 < n ? b.z : 0.f;
      b.w = j + 3 < n ? b.w : 0.f;
    }
    s0 += a.x * b.x + a.y * b.y;
    s1 += a.z * b.z + a.w * b.w;
  }
  return s0 + s1;
}

// two dots of one row (the row's loads shared): ox = r.x, oy = r.y
template <int NVP>
__device__ __forceinline__ void rowdot2_u(const float* r, const float* x, const float* y, int n, float& ox, float& oy) {
  float s0 = 0.f, s1 = 0.f, t0 = 0.f, t1 = 0.f;
#pragma unroll
  for (int j = 0; j < NVP; j += 4) {
    dot_chunk_barrier(j);
    const float4 a = *reinterpret_cast<const float4*>(r + j);
    float4 b = *reinterpret_cast<const float4*>(x + j);
    float4 c = *reinterpret_cast<const float4*>(y + j);
    if (j + 4 > n) {
      b.x = j < n ? b.x : 0.f; b.y = j + 1 < n ? b.y : 0.f; b.z = j + 2 < n ? b.z : 0.f; b.w = j + 3 < n ? b.w : 0.f;
      c.x = j < n ? c.x : 0.f; c.y = j + 1 < n ? c.y : 0.f; c.z = j + 2 < n ? c.z : 0.f; c.w = j + 3 < n ? c.w : 0.f;
    }
    s0 += a.x * b.x + a.y * b.y;
    s1 += a.z * b.z + a.w * b.w;
    t0 += a.x * c.x + a.y * c.y;
    t1 += a.z * c.z + a.w * c.w;
  }
  ox = s0 + s1;
  oy = t0 + t1;
}

// y = A x for the full symmetric (zero-padded) A, one row per lane
template <int NT, int NVP>
__device__ __forceinline__ void symv_u(const float* A, int n, int ld, const float* x, float* y) {
  for (int i = (threadIdx.x & 63); i < n; i += NT) y[i] = rowdot_u<NVP>(A + i * ld, x, n);
}

// dot of an aligned row with an aligned vector (float4 loads, 2 accumulators)
__device__ __forceinline__ float rowdot(const float* r, const float* x, int n) {
  float s0 = 0.f, s1 = 0.f;
  int j = 0;
  for (; j + 4 <= n; j += 4) {
    const float4 a = *reinterpret_cast<const float4*>(r + j);
    const float4 b = *reinterpret_cast<const float4*>(x + j);
    s0 += a.x * b.x + a.y * b.y;
    s1 += a.z * b.z + a.w * b.w;
  }
  for (; j < n; j++) s0 += r[j] * x[j];
  return s0 + s1;
}

// ---- register-resident LDL^T (lane i owns row i; NVP = padded size) ---------
#ifndef MJH_PK_FACTOR
#define MJH_PK_FACTOR 1
#endif
// Right-looking LDL^T fully unrolled over compile-time column indices: the
// entries of other rows come from v_readlane, so the factorisation never
// touches LDS between columns. Rows >= n are inert identity rows.
template <int NVP, bool PK>
__device__ __forceinline__ void load_row_lower(const float* A, int n, int ld, float (&a)[NVP]) {
  const int lane = threadIdx.x & 63;
  // a packed row's float4s beyond its length are the next rows' (scratch right
  // of the diagonal); the region holds lrow(NVP) words, so no read leaves it
  const float* r = A + lofs<PK>(lane < n ? lane : 0, ld);
#pragma unroll
  for (int k = 0; k < NVP; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(r + k);
    a[k] = v.x; a[k + 1] = v.y; a[k + 2] = v.z; a[k + 3] = v.w;
  }
  if (lane >= n) {
#pragma unroll
    for (int k = 0; k < NVP; k++) a[k] = (k == lane) ? 1.f : 0.f;
  }
}

// factor of the rows already in registers (lane i: row i, identity rows for
// lanes >= n); the factored rows are stored to A
template <int NVP, bool PK>
__device__ __forceinline__ void ldl_factor_rows(float (&a)[NVP], float* A, int n, int ld) {
  // Branch-free: lane i updates its whole row each step; entries right of the
  // diagonal are scratch never read back (only rdlane(a[k], j) with k < j, i.e.
  // lower-triangle values, crosses lanes), and rows >= n are identity rows, so
  // the padded steps k >= n are exact no-ops for rows < n.
  const int lane = threadIdx.x & 63;
  // the row update runs on pairs (v_pk_fma_f32: two entries per VALU issue);
  // a pair that starts at k only writes scratch a[k] (overwritten below for
  // rows >= k, right of the diagonal for rows < k)
  typedef float v2f __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int k = 0; k < NVP; k++) {
    const float ak = a[k];
    float piv = rdlane_f(ak, k);
    piv = piv < MJH_MINVAL ? MJH_MINVAL : piv;
    const float lik = ak * __builtin_amdgcn_rcpf(piv);  // v_rcp_f32 (1 ulp), not the IEEE division sequence
#if MJH_PK_FACTOR
    const v2f l2 = {lik, lik};
#pragma unroll
    for (int j = (k + 1) & ~1; j < NVP; j += 2) {
      const v2f r = {rdlane_f(ak, j), rdlane_f(ak, j + 1)};
      v2f x = {a[j], a[j + 1]};
      x -= l2 * r;
      a[j] = x.x;
      a[j + 1] = x.y;
    }
#else
#pragma unroll
    for (int j = k + 1; j < NVP; j++) a[j] -= lik * rdlane_f(ak, j);
#endif
    a[k] = lane > k ? lik : (lane == k ? piv : a[k]);
  }
  if (lane < n) {
    float* r = A + lofs<PK>(lane, ld);
    const int len = lspan<PK>(lane, ld);
#pragma unroll
    for (int k = 0; k < NVP; k += 4)
      if (k < len) *reinterpret_cast<float4*>(r + k) = make_float4(a[k], a[k + 1], a[k + 2], a[k + 3]);
  }
  wsync();
}

// M's rows (full rows of stride ldm >= NVP, 16-byte aligned, in global scratch) into
// A's rows: lane i issues all of row i's 16-byte loads before its stores. The
// element-strided copy this replaces (i += NT over n ldm entries) waited one global
// round trip per iteration: 21 in a row for G1's implicitfast integration.
template <int NVP, bool PK>
__device__ __forceinline__ void mass_rows_to(const float* M, float* A, int n, int ld) {
  const int lane = threadIdx.x & 63;
  wsync();
  if (lane < n) {
    float4 v[NVP / 4];
    const float* s = M + lane * ld;
#pragma unroll
    for (int k = 0; k < NVP; k += 4) v[k >> 2] = *reinterpret_cast<const float4*>(s + k);
    float* r = A + lofs<PK>(lane, ld);
    const int len = lspan<PK>(lane, ld);
#pragma unroll
    for (int k = 0; k < NVP; k += 4)
      if (k < len) *reinterpret_cast<float4*>(r + k) = v[k >> 2];
  }
  wsync();
}

template <int NVP, bool PK>
__device__ MJH_SOLVER_INLINE void ldl_factor_reg(float* A, int n, int ld) {
  float a[NVP];
  wsync();
  load_row_lower<NVP, PK>(A, n, ld, a);
  ldl_factor_rows<NVP, PK>(a, A, n, ld);
}

// The factor of the rows in A (as ldl_factor_reg) with the forward substitution
// of b (x, in LDS) carried through the same column sweep, then the backward
// substitution: x = (L D L^T)^-1 b in place. The same operations in the same
// order as ldl_factor_reg + ldl_solve_reg (bit-identical): the forward update
// of column k uses the multipliers the factor computes at step k, and y_k is
// final once the sweep reaches column k. Saves the solve's reload of the rows
// and its separate forward sweep (MJH_FUSED_FWD).
template <int NVP, bool PK>
__device__ MJH_SOLVER_INLINE void ldl_factor_solve_reg(float* A, int n, int ld, float* x) {
  const int lane = threadIdx.x & 63;
  float a[NVP];
  wsync();
  load_row_lower<NVP, PK>(A, n, ld, a);
  float xi = lane < n ? x[lane] : 0.f, di = 1.f;
  typedef float v2f __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int k = 0; k < NVP; k++) {
    const float ak = a[k];
    float piv = rdlane_f(ak, k);
    piv = piv < MJH_MINVAL ? MJH_MINVAL : piv;
    const float lik = ak * __builtin_amdgcn_rcpf(piv);
    const float xk = rdlane_f(xi, k);
    xi -= (lane > k ? lik : 0.f) * xk;
    di = lane == k ? piv : di;
#if MJH_PK_FACTOR
    const v2f l2 = {lik, lik};
#pragma unroll
    for (int j = (k + 1) & ~1; j < NVP; j += 2) {
      const v2f r = {rdlane_f(ak, j), rdlane_f(ak, j + 1)};
      v2f y = {a[j], a[j + 1]};
      y -= l2 * r;
      a[j] = y.x;
      a[j + 1] = y.y;
    }
#else
#pragma unroll
    for (int j = k + 1; j < NVP; j++) a[j] -= lik * rdlane_f(ak, j);
#endif
    a[k] = lane > k ? lik : (lane == k ? piv : a[k]);
  }
  if (lane < n) {
    float* r = A + lofs<PK>(lane, ld);
    const int len = lspan<PK>(lane, ld);
#pragma unroll
    for (int k = 0; k < NVP; k += 4)
      if (k < len) *reinterpret_cast<float4*>(r + k) = make_float4(a[k], a[k + 1], a[k + 2], a[k + 3]);
  }
  wsync();
  int cl = lane < n ? lane : 0;
  asm volatile("" : "+v"(cl));  // the column loads wait until the rows are dead
  float c[NVP];
#pragma unroll
  for (int k = 0; k < NVP; k++) c[k] = A[lofs<PK>(k < n ? k : 0, ld) + cl];
  xi = lane < n ? xi / di : 0.f;
#pragma unroll
  for (int k = NVP - 1; k > 0; k--) {
    const float xk = rdlane_f(xi, k);
    xi -= (lane < k && k < n ? c[k] : 0.f) * xk;
  }
  if (lane < n) x[lane] = xi;
  wsync();
}

// (L D L^T) x = b with the factor from ldl_factor_reg; x in LDS (in place).
template <int NVP, bool PK>
__device__ MJH_SOLVER_INLINE void ldl_solve_reg(const float* A, int n, int ld, float* x) {
  const int lane = threadIdx.x & 63;
  float a[NVP], c[NVP];
  wsync();
  load_row_lower<NVP, PK>(A, n, ld, a);  // L[i][k<i], D[i] at k == i
  int cl = lane < n ? lane : 0;
  float xi = lane < n ? x[lane] : 0.f;
  float di = 1.f;
#pragma unroll
  for (int k = 0; k < NVP; k++) {
    const float xk = rdlane_f(xi, k);
    xi -= (lane > k ? a[k] : 0.f) * xk;
    di = lane == k ? a[k] : di;
  }
  // the column loads wait until the row is dead (an opaque column index keeps
  // the compiler from hoisting them above the forward sweep): NVP live values
  // instead of 2 NVP
  asm volatile("" : "+v"(cl));
#pragma unroll
  for (int k = 0; k < NVP; k++) c[k] = A[lofs<PK>(k < n ? k : 0, ld) + cl];  // column i: L[k][i] (used for k > i)
  xi = lane < n ? xi / di : 0.f;
#pragma unroll
  for (int k = NVP - 1; k > 0; k--) {
    const float xk = rdlane_f(xi, k);
    xi -= (lane < k && k < n ? c[k] : 0.f) * xk;
  }
  if (lane < n) x[lane] = xi;
  wsync();
}

// y = A x for a symmetric matrix stored in full (16-byte aligned rows).
template <int NT>
__device__ MJH_SOLVER_INLINE void symv(const float* A, int n, int ld, const float* x, float* y) {
  for (int i = (threadIdx.x & 63); i < n; i += NT) {
    const float* r = A + i * ld;
    float s0 = 0.f, s1 = 0.f;
    int j = 0;
    for (; j + 4 <= n; j += 4) {
      const float4 a = *reinterpret_cast<const float4*>(r + j);
      const float4 b = *reinterpret_cast<const float4*>(x + j);
      s0 += a.x * b.x + a.y * b.y;
      s1 += a.z * b.z + a.w * b.w;
    }
    for (; j < n; j++) s0 += r[j] * x[j];
    y[i] = s0 + s1;
  }
}

// ---- contact primitives ----------------------------------------------------
struct Con {
  float dist, pos[3], frame[6];  // frame: normal + tangent hint
};

__device__ __forceinline__ int sphere_sphere(Con* c, float margin, const float* p1, float r1, const float* p2, float r2) {
  float dif[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  float cd = sqrtf(dot3(dif, dif));
  if (cd > margin + r1 + r2) return 0;
  float n[3];
  if (cd < MJH_MINVAL) {
    n[0] = 1.f; n[1] = 0.f; n[2] = 0.f;
  } else {
    float inv = 1.f / cd;
    n[0] = dif[0] * inv; n[1] = dif[1] * inv; n[2] = dif[2] * inv;
  }
  c->dist = cd - r1 - r2;
  float s = r1 + 0.5f * c->dist;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    c->pos[k] = p1[k] + n[k] * s;
    c->frame[k] = n[k];
    c->frame[3 + k] = 0.f;
  }
  return 1;
}

__device__ __forceinline__ int plane_sphere(Con* c, float margin, const float* pp, const float* pm, const float* sp, float r) {
  float n[3] = {pm[2], pm[5], pm[8]};
  float dif[3] = {sp[0] - pp[0], sp[1] - pp[1], sp[2] - pp[2]};
  float cd = dot3(dif, n);
  if (cd > margin + r) return 0;
  c->dist = cd - r;
  float s = r + 0.5f * c->dist;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    c->pos[k] = sp[k] - n[k] * s;
    c->frame[k] = n[k];
    c->frame[3 + k] = 0.f;
  }
  return 1;
}

// near-ties in the box functions' discrete choices go to the earlier candidate
// unless the later wins by kBoxTie x the size scale (the oracle's BOX_TIE), so
// float32 and float64 choose alike
constexpr float kBoxTie = 1e-5f;
// ---- box pairs (sphere-box, capsule-box, box-box): the oracle's algorithms
// (oracle/oracle.c raw_sphere_box / raw_capsule_box / raw_box_box) in float32.
// Boxes: centre bp, rotation bm (row-major, column k = axis k), half sizes bs.
__device__ __forceinline__ void to_box(const float* bp, const float* bm, const float* p, float* o) {
  const float d[3] = {p[0] - bp[0], p[1] - bp[1], p[2] - bp[2]};
#pragma unroll
  for (int k = 0; k < 3; k++) o[k] = bm[k] * d[0] + bm[3 + k] * d[1] + bm[6 + k] * d[2];
}
__device__ __forceinline__ void from_box(const float* bm, const float* v, float* o) {
#pragma unroll
  for (int k = 0; k < 3; k++) o[k] = bm[3 * k] * v[0] + bm[3 * k + 1] * v[1] + bm[3 * k + 2] * v[2];
}

// sphere (geom1) - box (geom2): the box point nearest the centre; a centre
// inside leaves through the nearest face (MuJoCo Warp sphere_box)
__device__ __noinline__ int sphere_box(Con* c, float margin, const float* sp, float r, const float* bp, const float* bm,
                                       const float* bs) {
  float lc[3], cl[3], dif[3];
  to_box(bp, bm, sp, lc);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    cl[k] = clampf(lc[k], -bs[k], bs[k]);
    dif[k] = cl[k] - lc[k];
  }
  const float dist = sqrtf(dot3(dif, dif));
  if (dist - r > margin) return 0;
  float nl[3] = {0.f, 0.f, 0.f}, pl[3];
  if (dist <= MJH_MINVAL) {
    float closest = 2.f * (bs[0] + bs[1] + bs[2]);
    const float tie = kBoxTie * (bs[0] + bs[1] + bs[2]);
    int kf = 0;
    for (int i = 0; i < 6; i++) {
      const float fd = fabsf((i & 1 ? 1.f : -1.f) * bs[i >> 1] - lc[i >> 1]);
      if (closest > fd + tie) { closest = fd; kf = i; }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) nl[k] = k == (kf >> 1) ? (kf & 1 ? -1.f : 1.f) : 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) pl[k] = lc[k] + nl[k] * (r - closest) * 0.5f;
    c->dist = -closest - r;
  } else {
#pragma unroll
    for (int k = 0; k < 3; k++) nl[k] = dif[k] / dist;
#pragma unroll
    for (int k = 0; k < 3; k++) pl[k] = 0.5f * (cl[k] + lc[k] + nl[k] * r);
    c->dist = dist - r;
  }
  float pw[3], nw[3];
  from_box(bm, pl, pw);
  from_box(bm, nl, nw);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    c->pos[k] = bp[k] + pw[k];
    c->frame[k] = nw[k];
    c->frame[3 + k] = 0.f;
  }
  return 1;
}

__device__ __forceinline__ float box_sdf(const float* bs, const float* q) {
  float out = 0.f, in = -1e30f;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float o = fabsf(q[k]) - bs[k], e = fmaxf(o, 0.f);
    out += e * e;
    in = fmaxf(in, o);
  }
  return out > 0.f ? sqrtf(out) : in;
}

// capsule (geom1) - box (geom2): both segment ends as spheres when both touch,
// otherwise one sphere at the segment point nearest the box (golden section on
// the convex signed distance, 40 steps)
__device__ __noinline__ int capsule_box(Con* out, float margin, const float* cp, const float* ax, float h, float r,
                                        const float* bp, const float* bm, const float* bs) {
  float a[3], b[3];
#pragma unroll
  for (int k = 0; k < 3; k++) { a[k] = cp[k] + ax[k] * h; b[k] = cp[k] - ax[k] * h; }
  Con ca, cb;
  const int na = sphere_box(&ca, margin, a, r, bp, bm, bs), nb = sphere_box(&cb, margin, b, r, bp, bm, bs);
  if (na && nb) {
    out[0] = ca;
    out[1] = cb;
#pragma unroll
    for (int k = 0; k < 3; k++) { out[0].frame[3 + k] = ax[k]; out[1].frame[3 + k] = ax[k]; }
    return 2;
  }
  float la[3], lb[3], q[3];
  to_box(bp, bm, a, la);
  to_box(bp, bm, b, lb);
  const float g = 0.6180339887498949f;
  float lo = 0.f, hi = 1.f, x1 = hi - g * (hi - lo), x2 = lo + g * (hi - lo);
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x1;
  float f1 = box_sdf(bs, q);
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x2;
  float f2 = box_sdf(bs, q);
  for (int it = 0; it < 40; it++) {
    if (f1 <= f2) {
      hi = x2; x2 = x1; f2 = f1; x1 = hi - g * (hi - lo);
#pragma unroll
      for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x1;
      f1 = box_sdf(bs, q);
    } else {
      lo = x1; x1 = x2; f1 = f2; x2 = lo + g * (hi - lo);
#pragma unroll
      for (int k = 0; k < 3; k++) q[k] = la[k] + (lb[k] - la[k]) * x2;
      f2 = box_sdf(bs, q);
    }
  }
  const float t = 0.5f * (lo + hi);
  float p[3];
#pragma unroll
  for (int k = 0; k < 3; k++) p[k] = a[k] + (b[k] - a[k]) * t;
  const int n = sphere_box(out, margin, p, r, bp, bm, bs);
  if (n) {
#pragma unroll
    for (int k = 0; k < 3; k++) out[0].frame[3 + k] = ax[k];
  }
  return n;
}

// box (geom1) - box (geom2): separating axes (face axes preferred within 5 %),
// face: incident face clipped against the reference face's side planes (the
// deepest point, then up to 3 more, each farthest from those kept); edge-edge:
// closest points of the two support edges
__device__ __noinline__ int box_box(Con* out, float margin, const float* pa, const float* ma, const float* sa, const float* pb,
                                    const float* mb, const float* sb) {
  float A[3][3], B[3][3];
  const float d[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { A[i][k] = ma[3 * k + i]; B[i][k] = mb[3 * k + i]; }
  float best = 1e30f, bn[3] = {0.f, 0.f, 0.f};
  const float tie = kBoxTie * (sa[0] + sa[1] + sa[2] + sb[0] + sb[1] + sb[2]);
  int bk = -1;
  for (int k = 0; k < 15; k++) {
    float L[3];
    if (k < 3) { L[0] = A[k][0]; L[1] = A[k][1]; L[2] = A[k][2]; }
    else if (k < 6) { L[0] = B[k - 3][0]; L[1] = B[k - 3][1]; L[2] = B[k - 3][2]; }
    else cross3(L, A[(k - 6) / 3], B[(k - 6) % 3]);
    const float ln = sqrtf(dot3(L, L));
    if (ln < 1e-6f) continue;
    for (int q = 0; q < 3; q++) L[q] /= ln;
    float ra = 0.f, rb = 0.f;
    for (int i = 0; i < 3; i++) { ra += sa[i] * fabsf(dot3(A[i], L)); rb += sb[i] * fabsf(dot3(B[i], L)); }
    const float dl = dot3(d, L), ov = ra + rb - fabsf(dl);
    if (ov < -margin) return 0;
    const float score = k < 6 ? ov : ov * 1.05f + 1e-9f;
    if (score < best - tie) {
      best = score;
      bk = k;
      for (int q = 0; q < 3; q++) bn[q] = dl < 0.f ? -L[q] : L[q];
    }
  }
  if (bk < 0) return 0;
  if (bk < 6) {
    const bool refA = bk < 3;
    const float *rp = refA ? pa : pb, *ip = refA ? pb : pa, *rs = refA ? sa : sb, *is = refA ? sb : sa;
    float R[3][3], I[3][3];
    for (int i = 0; i < 3; i++)
      for (int k = 0; k < 3; k++) { R[i][k] = refA ? A[i][k] : B[i][k]; I[i][k] = refA ? B[i][k] : A[i][k]; }
    float nr[3];
    for (int q = 0; q < 3; q++) nr[q] = refA ? bn[q] : -bn[q];
    const int ra = refA ? bk : bk - 3;
    int ia = 0;
    float mx = -1.f;
    for (int i = 0; i < 3; i++) {
      const float v = fabsf(dot3(I[i], nr));
      if (v > mx + kBoxTie) { mx = v; ia = i; }
    }
    const float isg = dot3(I[ia], nr) > 0.f ? -1.f : 1.f;
    float fc[3];
    for (int q = 0; q < 3; q++) fc[q] = ip[q] + I[ia][q] * is[ia] * isg;
    const int u = (ia + 1) % 3, v = (ia + 2) % 3;
    float poly[16][3], tmpp[16][3];
    int np = 4;
    for (int c = 0; c < 4; c++) {
      const float su = (c == 0 || c == 3) ? 1.f : -1.f, sv = (c < 2) ? 1.f : -1.f;
      for (int q = 0; q < 3; q++) poly[c][q] = fc[q] + I[u][q] * is[u] * su + I[v][q] * is[v] * sv;
    }
    for (int e = 0; e < 4 && np > 0; e++) {
      const int axis = e < 2 ? (ra + 1) % 3 : (ra + 2) % 3;
      const float sg = (e & 1) ? -1.f : 1.f;
      const float off = dot3(R[axis], rp) * sg + rs[axis];
      int nn = 0;
      for (int i = 0; i < np; i++) {
        const float* P = poly[i];
        const float* Q = poly[(i + 1) % np];
        const float dp = sg * dot3(R[axis], P) - off, dq = sg * dot3(R[axis], Q) - off;
        if (dp <= 0.f) { for (int q = 0; q < 3; q++) tmpp[nn][q] = P[q]; nn++; }
        if ((dp <= 0.f) != (dq <= 0.f)) {
          const float t = dp / (dp - dq);
          for (int q = 0; q < 3; q++) tmpp[nn][q] = P[q] + (Q[q] - P[q]) * t;
          nn++;
        }
      }
      np = nn;
      for (int i = 0; i < nn; i++)
        for (int q = 0; q < 3; q++) poly[i][q] = tmpp[i][q];
    }
    const float rfc = dot3(nr, rp) + rs[ra] * fabsf(dot3(R[ra], nr));
    float dep[16];
    int keep[16], nk = 0;
    for (int i = 0; i < np; i++) {
      dep[i] = dot3(nr, poly[i]) - rfc;
      if (dep[i] <= margin) keep[nk++] = i;
    }
    if (nk == 0) return 0;
    int sel[4], ns = 0, di = keep[0];
    for (int j = 1; j < nk; j++) if (dep[keep[j]] < dep[di] - tie) di = keep[j];
    sel[ns++] = di;
    while (ns < 4 && ns < nk) {
      int bj = -1;
      float bd = -1.f;
      for (int j = 0; j < nk; j++) {
        const int i = keep[j];
        bool used = false;
        float md = 1e30f;
        for (int s2 = 0; s2 < ns; s2++) {
          if (sel[s2] == i) used = true;
          const float dd[3] = {poly[i][0] - poly[sel[s2]][0], poly[i][1] - poly[sel[s2]][1], poly[i][2] - poly[sel[s2]][2]};
          md = fminf(md, sqrtf(dot3(dd, dd)));
        }
        if (!used && md > bd + tie) { bd = md; bj = i; }
      }
      if (bj < 0) break;
      sel[ns++] = bj;
    }
    for (int i = 0; i < ns; i++) {
      Con* c = out + i;
      c->dist = dep[sel[i]];
      for (int q = 0; q < 3; q++) {
        c->pos[q] = poly[sel[i]][q] - nr[q] * 0.5f * c->dist;
        c->frame[q] = bn[q];
        c->frame[3 + q] = 0.f;
      }
    }
    return ns;
  }
  const int ai = (bk - 6) / 3, bj = (bk - 6) % 3;
  float ca[3] = {pa[0], pa[1], pa[2]}, cb[3] = {pb[0], pb[1], pb[2]};
  for (int i = 0; i < 3; i++) {
    if (i != ai) {
      const float sg = dot3(A[i], bn) > 0.f ? 1.f : -1.f;
      for (int q = 0; q < 3; q++) ca[q] += A[i][q] * sa[i] * sg;
    }
    if (i != bj) {
      const float sg = dot3(B[i], bn) > 0.f ? -1.f : 1.f;
      for (int q = 0; q < 3; q++) cb[q] += B[i][q] * sb[i] * sg;
    }
  }
  const float w0[3] = {ca[0] - cb[0], ca[1] - cb[1], ca[2] - cb[2]};
  const float aa = dot3(A[ai], A[ai]), ab = dot3(A[ai], B[bj]), bb = dot3(B[bj], B[bj]);
  const float da = dot3(A[ai], w0), db = dot3(B[bj], w0), den = aa * bb - ab * ab;
  float s = den > 1e-12f ? (ab * db - bb * da) / den : 0.f;
  s = clampf(s, -sa[ai], sa[ai]);
  float t = clampf((ab * s + db) / bb, -sb[bj], sb[bj]);
  s = clampf((ab * t - da) / aa, -sa[ai], sa[ai]);
  float p1[3], p2[3];
  for (int q = 0; q < 3; q++) { p1[q] = ca[q] + A[ai][q] * s; p2[q] = cb[q] + B[bj][q] * t; }
  const float dd[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  const float dist = dot3(dd, bn);
  if (dist > margin) return 0;
  out[0].dist = dist;
  for (int q = 0; q < 3; q++) {
    out[0].pos[q] = 0.5f * (p1[q] + p2[q]);
    out[0].frame[q] = bn[q];
    out[0].frame[3 + q] = 0.f;
  }
  return 1;
}

// plane (geom1) - cylinder (geom2): the oracle's raw_plane_cylinder (MuJoCo
// mjc_PlaneCylinder) in float32: nearer-cap and farther-cap rim points, then
// the nearer cap's rim points 120 degrees either side of the first
__device__ __noinline__ int plane_cylinder(Con* out, float margin, const float* pp, const float* pm, const float* cp,
                                           const float* cm, float r, float h) {
  const float n[3] = {pm[2], pm[5], pm[8]};
  float ax[3] = {cm[2], cm[5], cm[8]};
  float prjaxis = dot3(n, ax);
  if (prjaxis > 0.f) {
#pragma unroll
    for (int k = 0; k < 3; k++) ax[k] = -ax[k];
    prjaxis = -prjaxis;
  }
  const float dif[3] = {cp[0] - pp[0], cp[1] - pp[1], cp[2] - pp[2]};
  const float dist0 = dot3(dif, n);
  float vec[3];
#pragma unroll
  for (int k = 0; k < 3; k++) vec[k] = ax[k] * prjaxis - n[k];
  const float len = sqrtf(dot3(vec, vec));
  if (len < MJH_MINVAL) {
#pragma unroll
    for (int k = 0; k < 3; k++) vec[k] = cm[3 * k] * r;
  } else {
#pragma unroll
    for (int k = 0; k < 3; k++) vec[k] *= r / len;
  }
  const float prjvec = dot3(vec, n);
#pragma unroll
  for (int k = 0; k < 3; k++) ax[k] *= h;
  prjaxis *= h;
  int cnt = 0;
  for (int e = 0; e < 2; e++) {
    const float sg = e == 0 ? 1.f : -1.f, dist = dist0 + sg * prjaxis + prjvec;
    if (dist > margin) continue;
    Con* c = out + cnt++;
    c->dist = dist;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      c->pos[k] = cp[k] + vec[k] + sg * ax[k] - n[k] * 0.5f * dist;
      c->frame[k] = n[k];
      c->frame[3 + k] = 0.f;
    }
  }
  const float dist = dist0 + prjaxis - 0.5f * prjvec;
  if (dist <= margin) {
    float side[3];
    cross3(side, vec, ax);
    const float sl = sqrtf(dot3(side, side));
#pragma unroll
    for (int k = 0; k < 3; k++) side[k] = sl > MJH_MINVAL ? side[k] * (r * 0.8660254037844386f / sl) : 0.f;
    for (int e = 0; e < 2; e++) {
      const float sg = e == 0 ? 1.f : -1.f;
      Con* c = out + cnt++;
      c->dist = dist;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        c->pos[k] = cp[k] + ax[k] - 0.5f * vec[k] + sg * side[k] - n[k] * 0.5f * dist;
        c->frame[k] = n[k];
        c->frame[3 + k] = 0.f;
      }
    }
  }
  return cnt;
}

// plane (geom1) - ellipsoid (geom2): the support point against the normal
// (oracle raw_plane_ellipsoid, MuJoCo Warp plane_ellipsoid)
__device__ __noinline__ int plane_ellipsoid(Con* c, float margin, const float* pp, const float* pm, const float* ep,
                                            const float* em, const float* s) {
  const float n[3] = {pm[2], pm[5], pm[8]};
  float nl[3], u[3], pl[3], pw[3];
#pragma unroll
  for (int k = 0; k < 3; k++) nl[k] = em[k] * n[0] + em[3 + k] * n[1] + em[6 + k] * n[2];
#pragma unroll
  for (int k = 0; k < 3; k++) u[k] = s[k] * nl[k];
  const float ul = fmaxf(sqrtf(dot3(u, u)), MJH_MINVAL);
#pragma unroll
  for (int k = 0; k < 3; k++) pl[k] = -s[k] * u[k] / ul;
#pragma unroll
  for (int k = 0; k < 3; k++) pw[k] = em[3 * k] * pl[0] + em[3 * k + 1] * pl[1] + em[3 * k + 2] * pl[2];
  const float dif[3] = {ep[0] + pw[0] - pp[0], ep[1] + pw[1] - pp[1], ep[2] + pw[2] - pp[2]};
  const float dist = dot3(dif, n);
  if (dist > margin) return 0;
  c->dist = dist;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    c->pos[k] = ep[k] + pw[k] - n[k] * 0.5f * dist;
    c->frame[k] = n[k];
    c->frame[3 + k] = 0.f;
  }
  return 1;
}

// sphere (geom1) - cylinder (geom2): side, cap or rim (oracle
// raw_sphere_cylinder, MuJoCo Warp sphere_cylinder)
__device__ __noinline__ int sphere_cylinder(Con* c, float margin, const float* sp, float rs, const float* cp, const float* cm,
                                            float r, float h) {
  const float ax[3] = {cm[2], cm[5], cm[8]};
  const float v[3] = {sp[0] - cp[0], sp[1] - cp[1], sp[2] - cp[2]};
  const float x = dot3(v, ax);
  float pr[3];
#pragma unroll
  for (int k = 0; k < 3; k++) pr[k] = v[k] - ax[k] * x;
  const float pr2 = dot3(pr, pr);
  bool side = fabsf(x) < h, cap = pr2 < r * r;
  if (side && cap) {
    if (h - fabsf(x) < r - sqrtf(pr2)) side = false; else cap = false;
  }
  if (side) {
    const float q[3] = {cp[0] + ax[0] * x, cp[1] + ax[1] * x, cp[2] + ax[2] * x};
    return sphere_sphere(c, margin, sp, rs, q, r);
  }
  const float sg = x > 0.f ? 1.f : -1.f;
  if (cap) {
    float nrm[3], d[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      nrm[k] = -sg * ax[k];
      d[k] = sp[k] - (cp[k] + sg * ax[k] * h);
    }
    const float dist = -dot3(d, nrm) - rs;
    if (dist > margin) return 0;
    c->dist = dist;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      c->pos[k] = sp[k] + nrm[k] * (rs + 0.5f * dist);
      c->frame[k] = nrm[k];
      c->frame[3 + k] = 0.f;
    }
    return 1;
  }
  const float prl = sqrtf(pr2);
  float q[3];
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = cp[k] + sg * ax[k] * h + (prl > MJH_MINVAL ? pr[k] * (r / prl) : 0.f);
  return sphere_sphere(c, margin, sp, rs, q, 0.f);
}

// Joint limit of a limited joint (mj_instantiateLimit): true if active, with
// pos = distance - margin and, for hinge/slide, sgn = +1 at the lower bound, -1
// at the upper. Ball: the rotation angle of the joint's quaternion against the
// larger range bound (the row's Jacobian is -(unit rotation axis)).
__device__ __forceinline__ bool joint_limit(int t, const float* q, const float* rng, float margin, float* pos, float* sgn) {
  if (t == 2 || t == 3) {
    const float dlo = q[0] - rng[0], dhi = rng[1] - q[0];
    *pos = fminf(dlo, dhi) - margin;
    *sgn = dlo < dhi ? 1.f : -1.f;
    return *pos < 0.f;
  }
  if (t == 1) {
    float r[3];
    const float ang = fabsf(quat2vel(r, q));
    *pos = fmaxf(rng[0], rng[1]) - ang - margin;
    *sgn = 1.f;
    return *pos < 0.f;
  }
  return false;
}

// the general convex pairs (sphere-ellipsoid, capsule-{ellipsoid,cylinder},
// ellipsoid-{ellipsoid,cylinder,box}, cylinder-{cylinder,box}): GJK + EPA and
// a Newton polish of the normal, one contact (mjh_convex.h, the oracle's
// collide() compiles the same source in float64)
__device__ __noinline__ int convex_pair(Con* c, int t1, const float* p1, const float* m1, const float* s1, int t2,
                                        const float* p2, const float* m2, const float* s2, float margin) {
  float n[3];
  if (!cvx_collide(t1, p1, m1, s1, t2, p2, m2, s2, margin, &c->dist, c->pos, n)) return 0;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    c->frame[k] = n[k];
    c->frame[3 + k] = 0.f;
  }
  return 1;
}

// Narrowphase for one pair (types ascending). Up to 4 contacts. `boxes`: the
// model has pairs that need the box, cylinder, ellipsoid or convex functions
// (Sizes::nboxpair; a compile-time
// 0 in the model-specialised instances of models without such pairs, whose
// code then carries none of them).
__device__ MJH_COLL_INLINE int narrowphase(int t1, int t2, const float* p1, const float* m1, const float* s1, const float* p2,
                           const float* m2, const float* s2, float margin, Con* out, bool boxes) {
  if (boxes && (t2 == 4 || t2 == 5)) {
    if (t1 == 0 && t2 == 4) return plane_ellipsoid(out, margin, p1, m1, p2, m2, s2);
    if (t1 == 0 && t2 == 5) return plane_cylinder(out, margin, p1, m1, p2, m2, s2[0], s2[1]);
    if (t1 == 2 && t2 == 5) return sphere_cylinder(out, margin, p1, s1[0], p2, m2, s2[0], s2[1]);
    if (t1 >= 2) return convex_pair(out, t1, p1, m1, s1, t2, p2, m2, s2, margin);
    return 0;
  }
  if (boxes && t2 == 6 && t1 >= 2) {
    if (t1 == 2) return sphere_box(out, margin, p1, s1[0], p2, m2, s2);
    if (t1 == 3) {
      const float ax[3] = {m1[2], m1[5], m1[8]};
      return capsule_box(out, margin, p1, ax, s1[1], s1[0], p2, m2, s2);
    }
    if (t1 == 6) return box_box(out, margin, p1, m1, s1, p2, m2, s2);
    return convex_pair(out, t1, p1, m1, s1, t2, p2, m2, s2, margin);
  }
  if (t1 == 0 && t2 == 2) return plane_sphere(out, margin, p1, m1, p2, s2[0]);
  if (t1 == 0 && t2 == 3) {
    float ax[3] = {m2[2], m2[5], m2[8]};
    float a[3], b[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      a[k] = p2[k] + ax[k] * s2[1];
      b[k] = p2[k] - ax[k] * s2[1];
    }
    int n1 = plane_sphere(out, margin, p1, m1, a, s2[0]);
    int n2 = plane_sphere(out + n1, margin, p1, m1, b, s2[0]);
    if (n1) { out[0].frame[3] = ax[0]; out[0].frame[4] = ax[1]; out[0].frame[5] = ax[2]; }
    if (n2) { out[n1].frame[3] = ax[0]; out[n1].frame[4] = ax[1]; out[n1].frame[5] = ax[2]; }
    return n1 + n2;
  }
  if (t1 == 0 && t2 == 6) {
    float n[3] = {m1[2], m1[5], m1[8]};
    float dif[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    float dist = dot3(dif, n);
    int cnt = 0;
    for (int i = 0; i < 8 && cnt < 4; i++) {
      float v[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 3; k++) {
        float s = (i & (1 << k)) ? s2[k] : -s2[k];
        v[0] += m2[k] * s;
        v[1] += m2[3 + k] * s;
        v[2] += m2[6 + k] * s;
      }
      float ld = dot3(n, v);
      if (dist + ld > margin) continue;
      Con* c = out + cnt++;
      c->dist = dist + ld;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        c->pos[k] = p2[k] + v[k] - n[k] * 0.5f * c->dist;
        c->frame[k] = n[k];
        c->frame[3 + k] = 0.f;
      }
    }
    return cnt;
  }
  if (t1 == 2 && t2 == 2) return sphere_sphere(out, margin, p1, s1[0], p2, s2[0]);
  if (t1 == 2 && t2 == 3) {
    float ax[3] = {m2[2], m2[5], m2[8]};
    float dif[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    float x = clampf(dot3(dif, ax), -s2[1], s2[1]);
    float v[3] = {p2[0] + ax[0] * x, p2[1] + ax[1] * x, p2[2] + ax[2] * x};
    return sphere_sphere(out, margin, p1, s1[0], v, s2[0]);
  }
  if (t1 == 3 && t2 == 3) {
    float a1[3] = {m1[2] * s1[1], m1[5] * s1[1], m1[8] * s1[1]};
    float a2[3] = {m2[2] * s2[1], m2[5] * s2[1], m2[8] * s2[1]};
    float dif[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    float ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    float u = -dot3(a1, dif), v = dot3(a2, dif), det = ma * mc - mb * mb;
    float v1[3], v2[3];
    if (fabsf(det) >= MJH_MINVAL) {
      float x1 = (mc * u - mb * v) / det, x2 = (ma * v - mb * u) / det;
      if (x1 > 1.f) { x1 = 1.f; x2 = (v - mb) / mc; }
      else if (x1 < -1.f) { x1 = -1.f; x2 = (v + mb) / mc; }
      if (x2 > 1.f) { x2 = 1.f; x1 = clampf((u - mb) / ma, -1.f, 1.f); }
      else if (x2 < -1.f) { x2 = -1.f; x1 = clampf((u + mb) / ma, -1.f, 1.f); }
#pragma unroll
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
      return sphere_sphere(out, margin, v1, s1[0], v2, s2[0]);
    }
    int n = 0;
    for (int e = 0; e < 2 && n < 2; e++) {
      float x1 = e ? -1.f : 1.f;
      float x2 = clampf((v - mb * x1) / mc, -1.f, 1.f);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
      n += sphere_sphere(out + n, margin, v1, s1[0], v2, s2[0]);
    }
    for (int e = 0; e < 2 && n < 2; e++) {
      float x2 = e ? -1.f : 1.f;
      float x1 = clampf((u - mb * x2) / ma, -1.f, 1.f);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
      n += sphere_sphere(out + n, margin, v1, s1[0], v2, s2[0]);
    }
    return n;
  }
  return 0;
}

__device__ __forceinline__ void make_frame(float f[9]) {
  normalize3(f);
  if (sqrtf(dot3(f + 3, f + 3)) < 0.5f) {
    f[3] = f[4] = f[5] = 0.f;
    if (f[1] < 0.5f && f[1] > -0.5f) f[4] = 1.f; else f[5] = 1.f;
  }
  float d = dot3(f, f + 3);
  f[3] -= d * f[0]; f[4] -= d * f[1]; f[5] -= d * f[2];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

// ---- constraint row parameters (solref/solimp -> D, aref) -------------------
__device__ __forceinline__ void row_params(float timestep, float pos_aref, float pos_imp, float invweight,
                                           const float* solref, const float* solimp, float jqvel, float* D,
                                           float* R, float* aref) {
  float timeconst = solref[0], dampratio = solref[1];
  if (solref[0] > 0.f && timeconst < 2.f * timestep) timeconst = 2.f * timestep;
  float dmin = clampf(solimp[0], MJH_MINIMP, MJH_MAXIMP);
  float dmax = clampf(solimp[1], MJH_MINIMP, MJH_MAXIMP);
  float width = fmaxf(solimp[2], MJH_MINVAL);
  float mid = clampf(solimp[3], MJH_MINIMP, MJH_MAXIMP);
  float power = fmaxf(solimp[4], 1.f);
  float k = 1.f / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  float b = 2.f / (dmax * timeconst);
  if (solref[0] <= 0.f) k = -solref[0] / (dmax * dmax);
  if (solref[1] <= 0.f) b = -solref[1] / dmax;
  float x = fabsf(pos_imp) / width, imp;
  if (x > 1.f) {
    imp = dmax;
  } else {
    float y = x < mid ? powf(x, power) / powf(mid, power - 1.f)
                      : 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
    imp = clampf(dmin + y * (dmax - dmin), dmin, dmax);
  }
  float r = fmaxf(invweight * (1.f - imp) / imp, MJH_MINVAL);
  *R = r;
  *D = 1.f / r;
  *aref = -k * imp * pos_aref - b * jqvel;
}

// The position-dependent part of row_params: D, R, aref_pos = -k imp pos and
// the damping coefficient b; the velocity stage completes aref = aref_pos - b J qvel
__device__ __forceinline__ void row_params_pos(float timestep, float pos_aref, float pos_imp, float invweight,
                                               const float* solref, const float* solimp, float* D, float* R,
                                               float* arefp, float* bb) {
  float timeconst = solref[0], dampratio = solref[1];
  if (solref[0] > 0.f && timeconst < 2.f * timestep) timeconst = 2.f * timestep;
  float dmin = clampf(solimp[0], MJH_MINIMP, MJH_MAXIMP);
  float dmax = clampf(solimp[1], MJH_MINIMP, MJH_MAXIMP);
  float width = fmaxf(solimp[2], MJH_MINVAL);
  float mid = clampf(solimp[3], MJH_MINIMP, MJH_MAXIMP);
  float power = fmaxf(solimp[4], 1.f);
  float k = 1.f / (dmax * dmax * timeconst * timeconst * dampratio * dampratio);
  float b = 2.f / (dmax * timeconst);
  if (solref[0] <= 0.f) k = -solref[0] / (dmax * dmax);
  if (solref[1] <= 0.f) b = -solref[1] / dmax;
  float x = fabsf(pos_imp) / width, imp;
  if (x > 1.f) {
    imp = dmax;
  } else {
    float y = x < mid ? powf(x, power) / powf(mid, power - 1.f)
                      : 1.f - powf(1.f - x, power) / powf(1.f - mid, power - 1.f);
    imp = clampf(dmin + y * (dmax - dmin), dmin, dmax);
  }
  float r = fmaxf(invweight * (1.f - imp) / imp, MJH_MINVAL);
  *R = r;
  *D = 1.f / r;
  *arefp = -k * imp * pos_aref;
  *bb = b;
}

// constraint state at jaref: writes force, returns Hessian weight (0 if inactive/linear)
__device__ __forceinline__ float row_state(int type, float D, float R, float fl, float jaref, float* force, float* cost) {
  if (type == MJH_CNSTR_FRICTION_DOF) {
    if (jaref >= R * fl) { *force = -fl; *cost = fl * jaref - 0.5f * R * fl * fl; return 0.f; }
    if (jaref <= -R * fl) { *force = fl; *cost = -fl * jaref - 0.5f * R * fl * fl; return 0.f; }
    *force = -D * jaref; *cost = 0.5f * D * jaref * jaref; return D;
  }
  if (jaref < 0.f) { *force = -D * jaref; *cost = 0.5f * D * jaref * jaref; return D; }
  *force = 0.f; *cost = 0.f; return 0.f;
}

// ---- elliptic cones (opt.cone == mjCONE_ELLIPTIC; generic instances only) ----
// A contact's dim rows (normal, then the frame's tangents / torsion / rolling)
// are evaluated together (MuJoCo Warp solver.py _update_constraint_efc,
// CONTACT_ELLIPTIC; oracle/oracle.c cone_eval): U0 = mu jar0, Uj = s_j jarj with
// the row scales s in efc_fl (mu = friction0 / sqrt(impratio), then
// friction_{j-1}), N = U0, T = |U1..|. Top zone (N >= mu T): free; bottom zone
// (mu N + T <= 0): every row quadratic; else the cone, cost 0.5 Dm (N - mu T)^2,
// Dm = D0 / (mu^2 (1 + mu^2)).
constexpr int kConeTop = 0, kConeBottom = 1, kConeMid = 2;
struct ConeRows {
  float jar[6], D[6], s[6];
};
// cost; forces f; zone; along a direction jv: *q2 = jv^T Hc jv (the cost's
// curvature, for the exact line search) when q2 != nullptr
__device__ __forceinline__ float cone_eval(int dim, const ConeRows& c, float (&f)[6], int* zone,
                                           const float* jv = nullptr, float* q2 = nullptr) {
  const float mu = c.s[0];
  float U[6], TT = 0.f;
  U[0] = c.jar[0] * mu;
#pragma unroll
  for (int j = 1; j < 6; j++) {
    U[j] = j < dim ? c.jar[j] * c.s[j] : 0.f;
    TT += U[j] * U[j];
  }
  const float N = U[0], T = TT > 0.f ? sqrtf(TT) : 0.f;
  if (N >= mu * T || (T <= 0.f && N >= 0.f)) {
#pragma unroll
    for (int j = 0; j < 6; j++) f[j] = 0.f;
    *zone = kConeTop;
    if (q2) *q2 = 0.f;
    return 0.f;
  }
  if (mu * N + T <= 0.f || (T <= 0.f && N < 0.f)) {
    float cost = 0.f, q = 0.f;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      f[j] = j < dim ? -c.D[j] * c.jar[j] : 0.f;
      cost += j < dim ? 0.5f * c.D[j] * c.jar[j] * c.jar[j] : 0.f;
      if (q2) q += j < dim ? c.D[j] * jv[j] * jv[j] : 0.f;
    }
    *zone = kConeBottom;
    if (q2) *q2 = q;
    return cost;
  }
  const float Dm = c.D[0] / fmaxf(mu * mu * (1.f + mu * mu), MJH_MINVAL), NmT = N - mu * T;
  f[0] = -Dm * NmT * mu;
#pragma unroll
  for (int j = 1; j < 6; j++) f[j] = j < dim ? -f[0] / T * U[j] * c.s[j] : 0.f;
  *zone = kConeMid;
  if (q2) {
    // w = S jv: jv^T Hc jv = Dm ((w0 - mu u.wt)^2 - (N - mu T) mu / T (|wt|^2 - (u.wt)^2)), u = Ut / T
    const float w0 = mu * jv[0];
    float uw = 0.f, ww = 0.f;
#pragma unroll
    for (int j = 1; j < 6; j++) {
      const float wj = j < dim ? c.s[j] * jv[j] : 0.f;
      uw += U[j] / T * wj;
      ww += wj * wj;
    }
    const float g = w0 - mu * uw;
    *q2 = Dm * (g * g - NmT * mu / T * (ww - uw * uw));
  }
  return 0.5f * Dm * NmT * NmT;
}

// ---- model specialisation -----------------------------------------------------
// A kernel instance with SPEC >= 0 takes the model sizes, the per-world layout
// and the model-image offsets as compile-time constants (mjh_spec_table.h,
// generated by tools/gen_spec.py from the benchmark models): every LDS/global
// scratch address folds into an instruction offset instead of living in
// (spilled) scalar registers. SPEC = -1 is the generic instance. The host picks
// a specialisation only when the model's launch plan matches it exactly.
// extension sensor groups (Sizes::sensor_ext_mask, spec/compiler.py SENSOR_EXT_GROUPS):
// the bits of the groups a model has; a specialised instance carries only their code
enum : int {
  kExtEnergy = 1, kExtForce = 2, kExtFramePos = 4, kExtFrameQuat = 8, kExtFrameVel = 16, kExtFrameAcc = 32,
  kExtLimit = 64, kExtActuator = 128, kExtBall = 256, kExtClock = 512, kExtRange = 1024, kExtMag = 2048
};
struct Sizes {
#define X_SZS(name) int name;
  MJH_MODEL_SIZES(X_SZS)
#undef X_SZS
};
constexpr int kSizeInts = sizeof(Sizes) / 4;
constexpr int kLayoutInts = sizeof(Layout) / 4;
constexpr int kImgInts = sizeof(ImgOff) / 4;
constexpr int kPlanInts = 1 + kSizeInts + kLayoutInts + kImgInts;

template <int K> __device__ __forceinline__ Sizes spec_sizes(const mjh_model& m) {
  Sizes z;
#define X_SZG(name) z.name = m.name;
  MJH_MODEL_SIZES(X_SZG)
#undef X_SZG
  return z;
}
// Word offsets (per world) of every data array inside one contiguous slab laid
// out in MJH_DATA_ARRAYS order, array f starting at nworld * offset(f): when the
// caller allocated the data that way (the Simulation does; checked on the host
// per launch), a specialised instance derives every data pointer from d.qpos
// with compile-time offsets instead of holding ~50 pointers in registers.
struct DataOff {
#define X_DOF(type, name, count) long long name;
  MJH_DATA_ARRAYS(X_DOF)
#undef X_DOF
};
__host__ __device__ __forceinline__ DataOff data_offsets(const Sizes& Z) {
#define X_DZ(name) const int name = Z.name;
  MJH_MODEL_SIZES(X_DZ)
#undef X_DZ
  DataOff o{};
  long long k = 0;
#define X_DO(type, name, count) o.name = k; k += ((count) > 1 ? (count) : 1);
  MJH_DATA_ARRAYS(X_DO)
#undef X_DO
  (void)nchain; (void)ncolgeom; (void)npair; (void)nsensor; (void)nmocap; (void)nconmax; (void)njmax; (void)na;
  (void)nsensordata; (void)nq; (void)nv; (void)nu; (void)nbody; (void)njnt; (void)ngeom; (void)nsite;
  return o;
}
template <int K> __device__ __forceinline__ Layout spec_layout(const Layout& a) { return a; }
template <int K> __device__ __forceinline__ ImgOff spec_imgoff(const ImgOff& a) { return a; }

// MJH_SPEC_TABLE: an alternative table (A/B builds of kernel variants whose
// launch plans differ, tools/build_variant.py)
#ifdef MJH_SPEC_TABLE
#include MJH_SPEC_TABLE
#else
#include "mjh_spec_table.h"
#endif

// ---- the step kernel --------------------------------------------------------
#ifndef MJH_PMINWAVES
#define MJH_PMINWAVES 1
#endif
#ifndef MJH_PRIO
#define MJH_PRIO -1  // -1: by model size (see the Newton loop)
#endif
#ifndef MJH_PERSIST
#define MJH_PERSIST 0
#endif
// resident worlds per CU for workgroups of fewer than 8 worlds (one-world
// workgroups: MJH_WPCU / 4 waves per SIMD); it sets the launch bound's wave
// target (the VGPR budget: 8 -> 256, 12 -> 168, 16 -> 128) and the per-world
// LDS budget alike
#ifndef MJH_MINWAVES
#define MJH_MINWAVES(wpb) ((wpb) < 8 ? MJH_WPCU / 4 : 1)
#endif
// MODE 0: the whole step in one launch. MODE 1: the position stage only
// (kinematics, com, CRB, M and its factor, collision, constraint rows and their
// position-dependent parameters), results to the global handoff region; a world
// whose qpos, mocap poses and model are unchanged since its last position pass
// (reuse != 0) exits at once: the pass's results are still in its scratch.
// MODE 2: everything else (velocity stage, solver, sensors, outputs,
// integration), starting from the handoff region. Split, the position stage
// needs far fewer registers and LDS, so it runs at higher occupancy, and the
// first physics step after a gated forward skips it.
// force / torque sensor (mj_sensorAcc after mj_rnePostConstraint): cfrc_int of
// the site's body sb -- over sb's subtree, I a + v x* I v minus the external
// wrench (xfrc_applied at the com; contact forces at the contact point, - on
// geom1's body and + on geom2's, the world body excluded), about the root's
// subtree com -- moved to the site and rotated into its frame; lane 0 writes
// out[3]. Out of line and recomputed per sensor: only models with these
// sensors call it, and inlined it would cost the step kernel registers on
// every path. Every lane of the wave calls it.
// ---- rays (mj_ray's primitive intersections): the distance along a unit ray
// to the geom's surface, -1 for no hit; a x^2 + 2 b x + c = 0 gives the
// smallest non-negative root. Out of line: only rangefinder models call it.
__device__ __forceinline__ float ray_quad(float a, float b, float c, float (&x)[2]) {
  float det = b * b - a * c;
  if (det < MJH_MINVAL) { x[0] = x[1] = -1.f; return -1.f; }
  det = sqrtf(det);
  x[0] = (-b - det) / a;
  x[1] = (-b + det) / a;
  return x[0] >= 0.f ? x[0] : (x[1] >= 0.f ? x[1] : -1.f);
}

__device__ __noinline__ float ray_geom(int type, const float* size, const float* pos, const float* mat, const float* pnt,
                                       const float* vec) {
  const float dif[3] = {pnt[0] - pos[0], pnt[1] - pos[1], pnt[2] - pos[2]};
  float lp[3], lv[3], xx[2];
  matT_vec(lp, mat, dif);
  matT_vec(lv, mat, vec);
  float x = -1.f, sol;
  switch (type) {
    case 0: {  // plane: from the front side, within the rendered rectangle when sized
      if (lv[2] > -MJH_MINVAL) return -1.f;
      x = -lp[2] / lv[2];
      if (x < 0.f) return -1.f;
      const float p0 = lp[0] + x * lv[0], p1 = lp[1] + x * lv[1];
      return ((size[0] <= 0.f || fabsf(p0) <= size[0]) && (size[1] <= 0.f || fabsf(p1) <= size[1])) ? x : -1.f;
    }
    case 2:
      return ray_quad(dot3(lv, lv), dot3(lv, lp), dot3(lp, lp) - size[0] * size[0], xx);
    case 3: {  // capsule: the round side between the flat ends, then the two caps
      sol = ray_quad(lv[0] * lv[0] + lv[1] * lv[1], lv[0] * lp[0] + lv[1] * lp[1],
                     lp[0] * lp[0] + lp[1] * lp[1] - size[0] * size[0], xx);
      if (sol >= 0.f && fabsf(lp[2] + sol * lv[2]) <= size[1]) x = sol;
      for (int side = -1; side <= 1; side += 2) {
        const float ld[3] = {lp[0], lp[1], lp[2] - side * size[1]};
        ray_quad(dot3(lv, lv), dot3(lv, ld), dot3(ld, ld) - size[0] * size[0], xx);
        for (int i = 0; i < 2; i++)
          if (xx[i] >= 0.f && side * (lp[2] + xx[i] * lv[2]) >= size[1] && (x < 0.f || xx[i] < x)) x = xx[i];
      }
      return x;
    }
    case 4: {  // ellipsoid
      float a = 0.f, b = 0.f, c = -1.f;
      for (int i = 0; i < 3; i++) {
        const float si = 1.f / (size[i] * size[i]);
        a += si * lv[i] * lv[i]; b += si * lv[i] * lp[i]; c += si * lp[i] * lp[i];
      }
      return ray_quad(a, b, c, xx);
    }
    case 5: {  // cylinder: the flat faces within the radius, then the round side
      if (fabsf(lv[2]) > MJH_MINVAL)
        for (int side = -1; side <= 1; side += 2) {
          sol = (side * size[1] - lp[2]) / lv[2];
          if (sol < 0.f) continue;
          const float p0 = lp[0] + sol * lv[0], p1 = lp[1] + sol * lv[1];
          if (p0 * p0 + p1 * p1 <= size[0] * size[0] && (x < 0.f || sol < x)) x = sol;
        }
      sol = ray_quad(lv[0] * lv[0] + lv[1] * lv[1], lv[0] * lp[0] + lv[1] * lp[1],
                     lp[0] * lp[0] + lp[1] * lp[1] - size[0] * size[0], xx);
      if (sol >= 0.f && fabsf(lp[2] + sol * lv[2]) <= size[1] && (x < 0.f || sol < x)) x = sol;
      return x;
    }
    case 6:  // box: the six faces
      for (int i = 0; i < 3; i++) {
        if (fabsf(lv[i]) <= MJH_MINVAL) continue;
        for (int side = -1; side <= 1; side += 2) {
          sol = (side * size[i] - lp[i]) / lv[i];
          if (sol < 0.f) continue;
          const int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
          if (fabsf(lp[i1] + sol * lv[i1]) <= size[i1] && fabsf(lp[i2] + sol * lv[i2]) <= size[i2] && (x < 0.f || sol < x))
            x = sol;
        }
      }
      return x;
    default:
      return -1.f;
  }
}

#ifndef MJH_FT_ATTR
#define MJH_FT_ATTR __noinline__
#endif
__device__ MJH_FT_ATTR void force_torque_sensor(int tid, int nb, int ncon, int type, int sb, const float* spos,
                                              const float* smat, float cut, const float* cinert, const float* cacc,
                                              const float* cvel, const float* xipos, const float* subtree_com,
                                              const float* xfrc, const int* body_rootid, const int* geom_bodyid,
                                              const float* con_frame, const float* con_pos, const int* con_geom,
                                              const int* con_efcadr, const int* con_dim, const float* con_fric,
                                              const float* efc_force, bool ell, unsigned long long r_tmk, float* out) {
  const bool bl = tid < nb;
  float fb[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float rc[3] = {0.f, 0.f, 0.f};
  if (bl && tid > 0) {
    float t1[6], t2[6], t3[6];
    inert_vec(t1, cinert + 10 * tid, cacc + 6 * tid);
    inert_vec(t2, cinert + 10 * tid, cvel + 6 * tid);
    cross_force(t3, cvel + 6 * tid, t2);
    const float* xf = xfrc + 6 * tid;
    const float* c = subtree_com + 3 * body_rootid[tid];
    rc[0] = c[0]; rc[1] = c[1]; rc[2] = c[2];
    const float r[3] = {xipos[3 * tid] - c[0], xipos[3 * tid + 1] - c[1], xipos[3 * tid + 2] - c[2]};
    float rf[3];
    cross3(rf, r, xf);
    for (int k = 0; k < 3; k++) {
      fb[k] = t1[k] + t3[k] - (xf[3 + k] + rf[k]);
      fb[3 + k] = t1[3 + k] + t3[3 + k] - xf[k];
    }
  }
  for (int c0 = 0; c0 < ncon; c0 += 64) {  // lane = contact, then each contact broadcast to its bodies' lanes
    const int ci = c0 + tid;
    float Fw[3] = {0.f, 0.f, 0.f}, Tw[3] = {0.f, 0.f, 0.f}, cp[3] = {0.f, 0.f, 0.f};
    int b1 = 0, b2 = 0;
    if (ci < ncon) {
      float F[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // mj_contactForce, contact frame
      const int r0 = con_efcadr[ci];
      if (r0 >= 0) {
        const int cdm = con_dim[ci];
        if (cdm == 1) {
          F[0] = efc_force[r0];
        } else if (ell) {
          for (int k = 0; k < cdm && k < 6; k++) F[k] = efc_force[r0 + k];
        } else {
          for (int e = 0; e < 2 * (cdm - 1); e++) F[0] += efc_force[r0 + e];
          for (int k = 1; k < cdm && k < 6; k++) F[k] = con_fric[5 * ci + k - 1] * (efc_force[r0 + 2 * k - 2] - efc_force[r0 + 2 * k - 1]);
        }
      }
      matT_vec(Fw, con_frame + 9 * ci, F);
      matT_vec(Tw, con_frame + 9 * ci, F + 3);
      cp[0] = con_pos[3 * ci]; cp[1] = con_pos[3 * ci + 1]; cp[2] = con_pos[3 * ci + 2];
      b1 = geom_bodyid[con_geom[2 * ci]];
      b2 = geom_bodyid[con_geom[2 * ci + 1]];
    }
    const int cnt = min(64, ncon - c0);
    for (int k = 0; k < cnt; k++) {
      const int k1 = __builtin_amdgcn_readlane(b1, k), k2 = __builtin_amdgcn_readlane(b2, k);
      float f3[3], t3[3], p3[3];
      for (int e = 0; e < 3; e++) { f3[e] = rl(Fw[e], k); t3[e] = rl(Tw[e], k); p3[e] = rl(cp[e], k); }
      const float sg = (tid == k2 ? 1.f : 0.f) - (tid == k1 ? 1.f : 0.f);
      if (bl && tid > 0 && sg != 0.f) {
        const float r[3] = {p3[0] - rc[0], p3[1] - rc[1], p3[2] - rc[2]};
        float t[3];
        cross3(t, r, f3);
        for (int e = 0; e < 3; e++) {
          fb[e] -= sg * (t3[e] + t[e]);
          fb[3 + e] -= sg * f3[e];
        }
      }
    }
  }
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = 1; k < nb; k++) {  // subtree sums, ascending k (as crb)
    const float in = (tid > 0 && ((rl64(r_tmk, k) >> tid) & 1ull)) ? 1.f : 0.f;
    for (int e = 0; e < 6; e++) acc[e] += in * rl(fb[e], k);
  }
  float f6[6];
  for (int e = 0; e < 6; e++) f6[e] = rl(acc[e], sb);
  if (tid == 0) {
    const float* c = subtree_com + 3 * body_rootid[sb];
    const float dif[3] = {spos[0] - c[0], spos[1] - c[1], spos[2] - c[2]};
    float t[3], v[3], o[3];
    cross3(t, dif, f6 + 3);
    if (type == 4) { v[0] = f6[3]; v[1] = f6[4]; v[2] = f6[5]; }
    else { v[0] = f6[0] - t[0]; v[1] = f6[1] - t[1]; v[2] = f6[2] - t[2]; }
    matT_vec(o, smat, v);
    for (int e = 0; e < 3; e++) out[e] = cut > 0.f ? clampf(o[e], -cut, cut) : o[e];
  }
}

template <int WPB, int NVP, int SPEC = -1, bool SLAB = false, int MODE = 0>
__global__ __launch_bounds__(64 * WPB, MODE == 1 ? MJH_PMINWAVES : MJH_MINWAVES(WPB)) void step_kernel(const mjh_model m, const mjh_data d, const Layout Lo_,
                                                         const ImgOff Io_, const unsigned char* gate, int reuse,
                                                         unsigned long long key, int step_flag) {
  constexpr int NT = 64;  // one wave per world
  const Layout Lo = spec_layout<SPEC>(Lo_);
  const ImgOff Io = spec_imgoff<SPEC>(Io_);
  const Sizes Z = spec_sizes<SPEC>(m);
  const DataOff DO = data_offsets(Z);
  char* const slab0 = reinterpret_cast<char*>(d.qpos);
  const long long nw4 = 4ll * d.nworld;
#define DP(name) (SLAB ? reinterpret_cast<decltype(d.name)>(slab + DO.name * nw4) : d.name)
  extern __shared__ float smem[];
  if (gate != nullptr && *gate == 0) return;  // gated forward: nothing to recompute
  constexpr bool IMG_GLOBAL = img_global(WPB);
  const float* const imgb = img_base<IMG_GLOBAL>(reinterpret_cast<const float*>(m.image), smem);
  const int kImgLds = IMG_GLOBAL ? 0 : Io.img_words;
  // shared model image -> LDS (whole workgroup, 16-byte coalesced)
  if constexpr (!IMG_GLOBAL) {
    const float4* src = reinterpret_cast<const float4*>(m.image);
    float4* dst = reinterpret_cast<float4*>(smem);
    for (int i = threadIdx.x; i < (Io.img_words >> 2); i += 64 * WPB) dst[i] = src[i];
    __syncthreads();
  }
  const int wave = threadIdx.x >> 6;
  // a checksum of the staged model image (each wave over the whole image: no
  // cross-wave exchange), part of the position-reuse snapshot, so an in-place
  // edit of a shared model field between a forward and a step is seen
  // (the fused kernel computes it only where it is compared or saved: a step
  // whose qpos / fields / key already match a saved snapshot, or a forward
  // saving one — not on the steps that integrated since the last forward)
  auto image_hash = [&]() -> unsigned long long {
    const uint4* iw = reinterpret_cast<const uint4*>(IMGB);
    unsigned h1 = 0u, h2 = 0u;
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < (Io.img_words >> 2); i += 64) {
      const uint4 v = iw[i];
      const unsigned k = 8u * (unsigned)i + 1u;
      h1 += v.x * k + v.y * (k + 2u) + v.z * (k + 4u) + v.w * (k + 6u);
      h2 += (v.x ^ 0x9E3779B9u) * 0x85EBCA6Bu + (v.y ^ k) * 0xC2B2AE35u + (v.z + k) * 0x27D4EB2Fu + (v.w ^ (k << 7)) * 0x165667B1u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      h1 += __shfl_xor(h1, o, 64);
      h2 += __shfl_xor(h2, o, 64);
    }
    return ((unsigned long long)h2 << 32) | h1;
  };
  unsigned long long img_hash = MODE == 1 ? image_hash() : 0ull;
  // MJH_PERSIST (fused kernel): one workgroup per resident slot, each wave
  // claims the next world (in the cost order below) from a counter the pack
  // launch zeroes, so a wave done with a cheap world starts another instead of
  // idling until its workgroup's slowest world is done
  constexpr bool PERSIST = MJH_PERSIST != 0 && MODE == 0;
  unsigned* const claim = reinterpret_cast<unsigned*>(m.image) + Io.img_words;
  for (;;) {
  int slot;
  if constexpr (PERSIST) {
    unsigned c = 0u;
    if ((threadIdx.x & 63) == 0) c = atomicAdd(claim, 1u);
    slot = __builtin_amdgcn_readfirstlane((int)c);
    if (slot >= d.nworld) return;
  } else {
    (void)claim;
    slot = blockIdx.x * WPB + wave;
    if (slot >= d.nworld) return;
  }
  // optional cost-sorted world order: a workgroup's worlds then take similar
  // time, so its LDS is not held hostage by one slow world (the position pass,
  // of nearly uniform cost, keeps the identity order)
  // wave-uniform: readfirstlane keeps w, the world bases and every pointer
  // derived from them in SGPRs (a vector load of world_order otherwise puts
  // ~20 64-bit scratch pointers in VGPR pairs, live across the whole step).
  // One-world workgroups only: the 8-world instance is not VGPR-bound and the
  // SGPR pairs spill there (Go1 0.551 -> 0.559 ms)
  // whole-CU workgroups take the cost order's ranks b, b + nblocks, ... so each
  // CU gets a mix of expensive and cheap worlds
  const int rank = (WPB > 1 && cu_worlds(WPB) && d.nworld % WPB == 0) ? wave * (int)gridDim.x + (int)blockIdx.x : slot;
  const int w0 = (MODE != 1 && d.world_order) ? (int)d.world_order[rank] : slot;
  const int w = cu_worlds(WPB) ? __builtin_amdgcn_readfirstlane(w0) : w0;
  const int tid = threadIdx.x & 63;
  // mj_step (integration) or mj_forward: a runtime flag, not a template
  // parameter, so both run the very same code up to the integration (a step
  // reusing a forward's position stage is then bit-identical to recomputing it)
  const bool STEP = step_flag != 0;
  // the world's LDS and data bases, made opaque per claimed world: otherwise
  // every address derived from them is hoisted out of the world loop and kept
  // live across it (register spills)
  int sofs = kImgLds + wave * (MODE == 1 ? Lo.ptotal : Lo.total);
  long long zofs = 0;
  if constexpr (PERSIST) asm volatile("" : "+v"(sofs), "+s"(zofs));
  char* const slab = slab0 + zofs;
  float* S = smem + sofs;
  int* SI = reinterpret_cast<int*>(S);
  float* G = d.scratch + (long long)w * d.scratch_words;  // this world's global scratch
  const long long W = w;
  const int nq = Z.nq, nv = Z.nv, nb = Z.nbody, nu = Z.nu, nj = Z.njnt;
  const int ldm = Lo.ldm, ldj = Lo.ldj;
  // the factor's rows: packed lower-triangular for one-world workgroups (the
  // split position launch hands the factor to the velocity launch, whose
  // workgroup shape decides the packing)
  constexpr bool PKL = pack_l(MODE == 1 ? wpb_of_nvp(NVP) : WPB);
  const int kLWords = PKL ? lrow(NVP) : nv * ldm;
  // elliptic friction cones: the generic instances only (the model-specialised
  // ones are picked for pyramidal cones), J in global scratch (virtual rows of
  // the cone Hessian after row rcap)
  const bool ELL = SPEC < 0 && Rg::J && m.cone == 1;

  constexpr bool HO = MODE == 1;
  float* qpos = HO ? S : SP(qpos);
  float* qvel = SP(qvel);
  float* qacc = SP(qacc);
  float* qacc_smooth = SP(qacc_smooth);
  float* qfrc_smooth = SP(qfrc_smooth);
  float* qfrc_bias = SP(qfrc_bias);
  float* qfrc_con = SP(qfrc_con);
  float* qfrc_passive = SP(qfrc_passive);
  // actuator forces per dof accumulate with LDS atomics in tmp2 (otherwise
  // unused); the global qfrc_act region stays reserved in the layout
  float* qfrc_act = SP(tmp2);
  float* grad = SP(grad);
  float* search = SP(search);
  float* Ma = SP(Ma);
  float* Mv = SP(Mv);
  float* tmp = SP(tmp);
  float* tmp2 = SP(tmp2);
  // slab data: the body and joint arrays the step outputs are computed in place in
  // the data arrays (this world's rows), not in global scratch copied out at the end
  constexpr bool kOutDirect = SLAB && MJH_OUT_DIRECT && Rg::xpos && Rg::xquat && Rg::xmat && Rg::xipos && Rg::ximat &&
                              Rg::subtree_com && Rg::cvel && Rg::cacc && Rg::xanchor && Rg::xaxis;
  const long long wb = W * Z.nbody, wj = W * Z.njnt;
  float* xpos = kOutDirect ? DP(xpos) + 3 * wb : SP(xpos);
  float* xquat = kOutDirect ? DP(xquat) + 4 * wb : SP(xquat);
  float* xmat = kOutDirect ? DP(xmat) + 9 * wb : SP(xmat);
  float* xipos = kOutDirect ? DP(xipos) + 3 * wb : SP(xipos);
  float* ximat = kOutDirect ? DP(ximat) + 9 * wb : SP(ximat);
  float* subtree_com = kOutDirect ? DP(subtree_com) + 3 * wb : SP(subtree_com);
  float* cinert = SP(cinert);
  float* crb = SP(crb);
  float* cvel = kOutDirect ? DP(cvel) + 6 * wb : SP(cvel);
  float* cacc = kOutDirect ? DP(cacc) + 6 * wb : SP(cacc);
  float* cfrc = SP(cfrc);
  float* xanchor = kOutDirect ? DP(xanchor) + 3 * wj : SP(xanchor);
  float* xaxis = kOutDirect ? DP(xaxis) + 3 * wj : SP(xaxis);
  float* cdof = SP(cdof);
  float* cdof_dot = SP(cdof_dot);
  float* cgpos = SP(cgpos);
  float* cgmat = SP(cgmat);
  // contacts and sites computed in place in the data arrays as well (slab layout)
  constexpr bool kOutDirect2 = kOutDirect && MJH_OUT_DIRECT2 && Rg::sxpos && Rg::sxmat && Rg::con_pos &&
                               Rg::con_frame && Rg::con_dist && Rg::con_fric && Rg::con_imargin && Rg::con_dim &&
                               Rg::con_geom && Rg::con_efcadr;
  const long long s_row0 = d.site_wstride ? W * d.site_wstride + d.site_off : W * Z.nsite;
  float* sxpos = kOutDirect2 ? (d.site_wstride ? d.site_xpos : DP(site_xpos)) + 3 * s_row0 : SP(sxpos);
  float* sxmat = kOutDirect2 ? (d.site_wstride ? d.site_xmat : DP(site_xmat)) + 9 * s_row0 : SP(sxmat);
  float* Mm = SP(M);
  float* Lm = HO ? G + Lo.h_L : SP(L);
  float* act_force = SP(act_force);
  const long long wc = W * Z.nconmax;
  float* con_pos = kOutDirect2 ? DP(contact_pos) + 3 * wc : SP(con_pos);
  float* con_frame = kOutDirect2 ? DP(contact_frame) + 9 * wc : SP(con_frame);
  float* con_dist = kOutDirect2 ? DP(contact_dist) + wc : SP(con_dist);
  float* con_fric = kOutDirect2 ? DP(contact_friction) + 5 * wc : SP(con_fric);
  float* con_solref = SP(con_solref);
  float* con_solimp = SP(con_solimp);
  float* con_imargin = kOutDirect2 ? DP(contact_includemargin) + wc : SP(con_imargin);
  int* con_dim = kOutDirect2 ? DP(contact_dim) + wc : SPI(con_dim);
  int* con_geom = kOutDirect2 ? DP(contact_geom) + 2 * wc : SPI(con_geom);
  int* con_efcadr = kOutDirect2 ? DP(contact_efc_address) + wc : SPI(con_efcadr);
  float* J = SP(J);
  float* efc_pos = SP(efc_pos);
  int* efc_id = SPI(efc_id);
  unsigned long long* efc_mask = reinterpret_cast<unsigned long long*>(SP(efc_mask));
  int* sidx = SPI(sidx);
  float* red = S + (MODE == 1 ? Lo.pred : Lo.red);
  int* redi = SI + (MODE == 1 ? Lo.pred : Lo.red) + 2 * (NT / 64) + 2;
  int* ints = SI + (MODE == 1 ? Lo.pints : Lo.ints);

  // per-world model fields (stride 0 = shared)
  const float* body_pos = WFIELD(body_pos);
  const float* body_quat = WFIELD(body_quat);
  const float* body_ipos = WFIELD(body_ipos);
  const float* body_iquat = WFIELD(body_iquat);
  const float* body_mass = WFIELD(body_mass);
  const float* body_inertia = WFIELD(body_inertia);
  const float* jnt_range = WFIELD(jnt_range);
  const float* jnt_stiffness = WFIELD(jnt_stiffness);
  const float* dof_armature = WFIELD(dof_armature);
  const float* dof_damping = WFIELD(dof_damping);
  const float* dof_frictionloss = WFIELD(dof_frictionloss);
  const float* geom_pos = WFIELD(geom_pos);
  const float* geom_quat = WFIELD(geom_quat);
  const float* geom_friction = WFIELD(geom_friction);
  const float* site_pos = WFIELD(site_pos);
  const float* site_quat = WFIELD(site_quat);
  const float* qpos0 = WFIELD(qpos0);

  (void)SI;

  // ---------------------------------------------------------------- load state
  for (int i = tid; i < nq; i += NT) qpos[i] = DP(qpos)[W * nq + i];
  if constexpr (MODE != 1)
    for (int i = tid; i < nv; i += NT) qvel[i] = DP(qvel)[W * nv + i];
  if (tid < I_COUNT) ints[tid] = (tid == I_MISC) ? 0x7fffffff : 0;
  wsync();
  // reuse snapshot: [valid, image hash (2 words), per-world model fields hash
  // (2), launch key (2: the host's hash of the model and data descriptors, so
  // option scalars and buffer addresses), qpos (nq), mocap pos/quat (7 nmocap)],
  // raw bits
  unsigned* const snap = reinterpret_cast<unsigned*>(G + Lo.h_snap);
  unsigned long long wf_hash = 0ull;
  // fused kernel: a step launch whose world is unchanged since the last
  // forward's position stage (which saved its LDS results, below) reuses them
  bool reused = false;
  if constexpr (MODE == 1 || MODE == 0) {
    {  // per-world (expanded) model fields of this world
      unsigned long long h = 0ull;
      int fid = 0;
#define X_DZ(name) const int name = Z.name;
      MJH_MODEL_SIZES(X_DZ)
#undef X_DZ
      (void)nchain; (void)ncolgeom; (void)npair; (void)nsensor; (void)nconmax; (void)njmax; (void)na; (void)nsensordata;
      (void)nu;
#define X_WH(type, name, count)                                                                                \
      if (m.name##_wstride) {                                                                                  \
        const unsigned* f = reinterpret_cast<const unsigned*>(m.name + W * m.name##_wstride);                  \
        for (int i = tid; i < (count); i += NT)                                                                \
          h += mix64(((unsigned long long)fid << 56) ^ ((unsigned long long)i << 32) ^ f[i]);                  \
      }                                                                                                        \
      fid++;
      MJH_MODEL_WARRAYS(X_WH)
#undef X_WH
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
      wf_hash = h;
    }
    if (reuse) {
      const unsigned* qb = reinterpret_cast<const unsigned*>(qpos);
      bool same = snap[0] == 1u && (MODE != 1 || (snap[1] == (unsigned)img_hash && snap[2] == (unsigned)(img_hash >> 32))) &&
                  snap[3] == (unsigned)wf_hash && snap[4] == (unsigned)(wf_hash >> 32) &&
                  snap[5] == (unsigned)key && snap[6] == (unsigned)(key >> 32);
      for (int i = tid; i < nq; i += NT) same = same && snap[7 + i] == qb[i];
      if (Z.nmocap > 0) {
        const unsigned* mp = reinterpret_cast<const unsigned*>(DP(mocap_pos) + W * Z.nmocap * 3);
        const unsigned* mq = reinterpret_cast<const unsigned*>(DP(mocap_quat) + W * Z.nmocap * 4);
        for (int i = tid; i < 3 * Z.nmocap; i += NT) same = same && snap[7 + nq + i] == mp[i];
        for (int i = tid; i < 4 * Z.nmocap; i += NT) same = same && snap[7 + nq + 3 * Z.nmocap + i] == mq[i];
      }
      if constexpr (MODE == 1) {
        if (__all(same)) return;  // the last position pass of this world is current
      } else if (STEP && __all(same)) {
        img_hash = image_hash();
        reused = snap[1] == (unsigned)img_hash && snap[2] == (unsigned)(img_hash >> 32);
      }
    }
  }
  // a fused launch that recomputes the position stage overwrites the arrays a
  // saved snapshot describes (a forward saves a new one at the end of its stage)
  if constexpr (MODE == 0) {
    if (!reused && tid == 0) snap[0] = 0u;
  }
  PROF(0);
#ifdef MJH_PROFILE
  if (tid == 0 && g_prof) {
    for (int k = 12; k < 20; k++) g_prof[(long long)w * 32 + k] = 0;
    g_prof[(long long)w * 32 + 30] = 0;
  }
#endif

  // ---------------------------------------------------------------- kinematics
  // Each lane walks its body's chain root->body (no per-level barriers). The
  // per-body normalisation matches a level-by-level sweep exactly.
  // nbody, nv <= 64 (mjh_model_check): lane b owns body b and lane i dof i, so
  // the tree phases below keep per-body / per-dof quantities in registers and
  // exchange them with v_readlane (uniform k) or ds_bpermute, instead of
  // serial chains of dependent global-scratch loads.
  const bool bl = tid < nb;
  // registers the velocity stage takes from the position stage (reloaded from
  // scratch by the split velocity kernel)
  float r_cin[10];
  float r_cdof[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int ncon = 0, nefc = 0;
  const unsigned long long* tmk = reinterpret_cast<const unsigned long long*>(IMG_L(body_treemask));
  const unsigned long long* dmk = reinterpret_cast<const unsigned long long*>(IMG_L(body_dofmask));
  // lane b holds body b's chain mask; the subtree loops read it by readlane
  // (no LDS load per body on their dependency chain)
  const unsigned long long r_tmk = bl ? tmk[tid] : 0ull;
  if (MODE == 1 || (MODE == 0 && !reused)) {
  float r_xipos[3] = {0.f, 0.f, 0.f}, r_ximat[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#ifdef MJH_KIN_CHAIN
  for (int b = tid; b < nb; b += NT) {
    float p[3] = {0.f, 0.f, 0.f}, q[4] = {1.f, 0.f, 0.f, 0.f};
    const int ca = IMG_I(body_chainadr)[b], cn = (b == 0) ? 0 : IMG_I(body_chainnum)[b];
    for (int c = 0; c < cn; c++) {
      const int k = IMG_I(body_chain)[ca + c];
      const int ja = IMG_I(body_jntadr)[k], jn = IMG_I(body_jntnum)[k];
      const int mid = Z.nmocap > 0 ? IMG_I(body_mocapid)[k] : -1;
      if (mid >= 0) {  // mocap body (a child of the world): pose from mocap_pos / mocap_quat
        const float* mp = DP(mocap_pos) + (W * Z.nmocap + mid) * 3;
        const float* mq = DP(mocap_quat) + (W * Z.nmocap + mid) * 4;
        p[0] = mp[0]; p[1] = mp[1]; p[2] = mp[2];
        q[0] = mq[0]; q[1] = mq[1]; q[2] = mq[2]; q[3] = mq[3];
        quat_normalize(q);
        continue;
      }
      if (jn == 1 && IMG_I(jnt_type)[ja] == 0) {
        const int qa = IMG_I(jnt_qposadr)[ja];
        p[0] = qpos[qa]; p[1] = qpos[qa + 1]; p[2] = qpos[qa + 2];
        q[0] = qpos[qa + 3]; q[1] = qpos[qa + 4]; q[2] = qpos[qa + 5]; q[3] = qpos[qa + 6];
        quat_normalize(q);
        if (k == b) {
          float R[9];
          quat2mat(R, q);
          xanchor[3 * ja] = p[0]; xanchor[3 * ja + 1] = p[1]; xanchor[3 * ja + 2] = p[2];
          xaxis[3 * ja] = R[2]; xaxis[3 * ja + 1] = R[5]; xaxis[3 * ja + 2] = R[8];
        }
        continue;
      }
      float R[9], t[3];
      quat2mat(R, q);
      mat_vec(t, R, body_pos + 3 * k);
      p[0] += t[0]; p[1] += t[1]; p[2] += t[2];
      quat_mul(q, q, body_quat + 4 * k);
      for (int j = ja; j < ja + jn; j++) {
        float Rq[9], ax[3], anc[3];
        quat2mat(Rq, q);
        mat_vec(ax, Rq, IMG_F(jnt_axis) + 3 * j);
        mat_vec(anc, Rq, IMG_F(jnt_pos) + 3 * j);
        anc[0] += p[0]; anc[1] += p[1]; anc[2] += p[2];
        const int qa = IMG_I(jnt_qposadr)[j];
        if (IMG_I(jnt_type)[j] == 2) {
          const float dd = qpos[qa] - qpos0[qa];
          p[0] += ax[0] * dd; p[1] += ax[1] * dd; p[2] += ax[2] * dd;
        } else if (IMG_I(jnt_type)[j] == 3) {
          float ql[4], v[3];
          axis_angle(ql, IMG_F(jnt_axis) + 3 * j, qpos[qa] - qpos0[qa]);
          quat_mul(q, q, ql);
          quat2mat(Rq, q);
          mat_vec(v, Rq, IMG_F(jnt_pos) + 3 * j);
          p[0] = anc[0] - v[0]; p[1] = anc[1] - v[1]; p[2] = anc[2] - v[2];
        } else if (IMG_I(jnt_type)[j] == 1) {  // ball: the normalised qpos quaternion, about the anchor
          float ql[4] = {qpos[qa], qpos[qa + 1], qpos[qa + 2], qpos[qa + 3]}, v[3];
          quat_normalize(ql);
          quat_mul(q, q, ql);
          quat2mat(Rq, q);
          mat_vec(v, Rq, IMG_F(jnt_pos) + 3 * j);
          p[0] = anc[0] - v[0]; p[1] = anc[1] - v[1]; p[2] = anc[2] - v[2];
        }
        if (k == b) {
          xanchor[3 * j] = anc[0]; xanchor[3 * j + 1] = anc[1]; xanchor[3 * j + 2] = anc[2];
          xaxis[3 * j] = ax[0]; xaxis[3 * j + 1] = ax[1]; xaxis[3 * j + 2] = ax[2];
        }
      }
      quat_normalize(q);
    }
#elif MJH_KIN_JUMP
  // Pointer jumping over the body tree: log2(depth) rounds instead of one round
  // per level. Each lane forms its body's transform relative to its parent (the
  // body offset, then its joints about their anchors: the chain walk's
  // operations in the parent's frame); round r composes it with the transform of
  // the ancestor 2^r levels up (ds_bpermute). The same poses as the level sweep
  // with the composition reassociated (float32 rounding differs).
  if (bl) {
    const int b = tid;
    float p[3] = {0.f, 0.f, 0.f}, q[4] = {1.f, 0.f, 0.f, 0.f};
    const int cn = b == 0 ? 0 : IMG_I(body_chainnum)[b];
    const int par = cn > 0 ? IMG_I(body_parentid)[b] : 0;
    const int ja = cn > 0 ? IMG_I(body_jntadr)[b] : 0, jn = cn > 0 ? IMG_I(body_jntnum)[b] : 0;
    const int mid = (cn > 0 && Z.nmocap > 0) ? IMG_I(body_mocapid)[b] : -1;
    const int jt0 = jn > 0 ? IMG_I(jnt_type)[ja] : -1, qa0 = jn > 0 ? IMG_I(jnt_qposadr)[ja] : 0;
    int anc = -1;  // the body whose frame (p, q) is expressed in (-1: the world)
    // joint j of the body applied to (p, q); anchor / axis in that frame
    auto apply_joint = [&](int j, float (&ax)[3], float (&an)[3]) {
      float jax[3], jp[3], Rq[9];
#pragma unroll
      for (int k = 0; k < 3; k++) { jax[k] = IMG_F(jnt_axis)[3 * j + k]; jp[k] = IMG_F(jnt_pos)[3 * j + k]; }
      const int jt = IMG_I(jnt_type)[j], qa = IMG_I(jnt_qposadr)[j];
      quat2mat(Rq, q);
      mat_vec(ax, Rq, jax);
      mat_vec(an, Rq, jp);
      an[0] += p[0]; an[1] += p[1]; an[2] += p[2];
      if (jt == 2) {
        const float dd = qpos[qa] - qpos0[qa];
        p[0] += ax[0] * dd; p[1] += ax[1] * dd; p[2] += ax[2] * dd;
      } else if (jt == 3 || jt == 1) {
        float ql[4], v[3];
        if (jt == 3) {
          axis_angle(ql, jax, qpos[qa] - qpos0[qa]);
        } else {
          ql[0] = qpos[qa]; ql[1] = qpos[qa + 1]; ql[2] = qpos[qa + 2]; ql[3] = qpos[qa + 3];
          quat_normalize(ql);
        }
        quat_mul(q, q, ql);
        quat2mat(Rq, q);
        mat_vec(v, Rq, jp);
        p[0] = an[0] - v[0]; p[1] = an[1] - v[1]; p[2] = an[2] - v[2];
      }
    };
    if (cn > 0) {
      if (mid >= 0) {  // mocap body (a child of the world): pose from mocap_pos / mocap_quat
        const float* mp = DP(mocap_pos) + (W * Z.nmocap + mid) * 3;
        const float* mq = DP(mocap_quat) + (W * Z.nmocap + mid) * 4;
        p[0] = mp[0]; p[1] = mp[1]; p[2] = mp[2];
        q[0] = mq[0]; q[1] = mq[1]; q[2] = mq[2]; q[3] = mq[3];
        quat_normalize(q);
      } else if (jn == 1 && jt0 == 0) {  // free joint: the pose is the joint's coordinates
        p[0] = qpos[qa0]; p[1] = qpos[qa0 + 1]; p[2] = qpos[qa0 + 2];
        q[0] = qpos[qa0 + 3]; q[1] = qpos[qa0 + 4]; q[2] = qpos[qa0 + 5]; q[3] = qpos[qa0 + 6];
        quat_normalize(q);
      } else {
#pragma unroll
        for (int k = 0; k < 3; k++) p[k] = body_pos[3 * b + k];
#pragma unroll
        for (int k = 0; k < 4; k++) q[k] = body_quat[4 * b + k];
        for (int j = ja; j < ja + jn; j++) {
          float ax[3], an[3];
          apply_joint(j, ax, an);
        }
        anc = par == 0 ? -1 : par;
      }
    }
    for (int r = 0; r < 6 && __any(anc >= 0); r++) {  // 2^6 levels >= any tree of <= 64 bodies
      const int src = anc >= 0 ? anc : b;
      float ap[3], aq[4];
#pragma unroll
      for (int k = 0; k < 3; k++) ap[k] = shfl(p[k], src);
#pragma unroll
      for (int k = 0; k < 4; k++) aq[k] = shfl(q[k], src);
      const int aa = __shfl(anc, src, 64);
      if (anc >= 0) {
        float Ra[9], t[3];
        quat2mat(Ra, aq);
        mat_vec(t, Ra, p);
        p[0] = ap[0] + t[0]; p[1] = ap[1] + t[1]; p[2] = ap[2] + t[2];
        quat_mul(q, aq, q);
        anc = aa;
      }
    }
    quat_normalize(q);
    // joint anchors and axes. A hinge's anchor and axis, and a slide's axis, are
    // fixed by the joint's own motion, so the body's final frame gives them; a
    // free joint's are its position and z axis. Ball joints and bodies with
    // several joints replay their joints from the parent's final pose.
    const bool replay = cn > 0 && mid < 0 && jn > 0 && !(jn == 1 && jt0 != 1);
    if (cn > 0 && mid < 0 && jn == 1 && jt0 != 1) {
      float R[9], ax[3], an[3], jax[3], jp[3];
      quat2mat(R, q);
      if (jt0 == 0) {
        an[0] = p[0]; an[1] = p[1]; an[2] = p[2];
        ax[0] = R[2]; ax[1] = R[5]; ax[2] = R[8];
      } else {
#pragma unroll
        for (int k = 0; k < 3; k++) { jax[k] = IMG_F(jnt_axis)[3 * ja + k]; jp[k] = IMG_F(jnt_pos)[3 * ja + k]; }
        mat_vec(ax, R, jax);
        mat_vec(an, R, jp);
        const float dd = jt0 == 2 ? qpos[qa0] - qpos0[qa0] : 0.f;
        an[0] += p[0] - ax[0] * dd; an[1] += p[1] - ax[1] * dd; an[2] += p[2] - ax[2] * dd;
      }
      xanchor[3 * ja] = an[0]; xanchor[3 * ja + 1] = an[1]; xanchor[3 * ja + 2] = an[2];
      xaxis[3 * ja] = ax[0]; xaxis[3 * ja + 1] = ax[1]; xaxis[3 * ja + 2] = ax[2];
    }
    if (__any(replay)) {
      float pp[3], pq[4];
#pragma unroll
      for (int k = 0; k < 3; k++) pp[k] = shfl(p[k], par);
#pragma unroll
      for (int k = 0; k < 4; k++) pq[k] = shfl(q[k], par);
      if (replay) {
        const float fp[3] = {p[0], p[1], p[2]}, fq[4] = {q[0], q[1], q[2], q[3]};
        float R[9], t[3], bp[3], bq[4];
#pragma unroll
        for (int k = 0; k < 3; k++) bp[k] = body_pos[3 * b + k];
#pragma unroll
        for (int k = 0; k < 4; k++) bq[k] = body_quat[4 * b + k];
        quat2mat(R, pq);
        mat_vec(t, R, bp);
        p[0] = pp[0] + t[0]; p[1] = pp[1] + t[1]; p[2] = pp[2] + t[2];
        quat_mul(q, pq, bq);
        for (int j = ja; j < ja + jn; j++) {
          float ax[3], an[3];
          apply_joint(j, ax, an);
          xanchor[3 * j] = an[0]; xanchor[3 * j + 1] = an[1]; xanchor[3 * j + 2] = an[2];
          xaxis[3 * j] = ax[0]; xaxis[3 * j + 1] = ax[1]; xaxis[3 * j + 2] = ax[2];
        }
        p[0] = fp[0]; p[1] = fp[1]; p[2] = fp[2];
        q[0] = fq[0]; q[1] = fq[1]; q[2] = fq[2]; q[3] = fq[3];
      }
    }
#else
  // Level-synchronous sweep: at level d the lanes of the bodies at depth d take
  // their parent's final pose from its lane (ds_bpermute) and apply their own
  // body offset and joints, whose inputs every lane loaded before the sweep. The
  // operations per body are those of a root-to-body chain walk; the chain of
  // dependent image loads per level is gone.
  if (bl) {
    const int b = tid;
    float p[3] = {0.f, 0.f, 0.f}, q[4] = {1.f, 0.f, 0.f, 0.f};
    const int cn = b == 0 ? 0 : IMG_I(body_chainnum)[b];  // depth (the chain ends at b)
    const int par = cn > 0 ? IMG_I(body_parentid)[b] : 0;
    const int ja = cn > 0 ? IMG_I(body_jntadr)[b] : 0, jn = cn > 0 ? IMG_I(body_jntnum)[b] : 0;
    const int mid = (cn > 0 && Z.nmocap > 0) ? IMG_I(body_mocapid)[b] : -1;
    const int jt0 = jn > 0 ? IMG_I(jnt_type)[ja] : -1, qa0 = jn > 0 ? IMG_I(jnt_qposadr)[ja] : 0;
    float bp[3] = {0.f, 0.f, 0.f}, bq[4] = {1.f, 0.f, 0.f, 0.f}, ax0[3] = {0.f, 0.f, 0.f}, jp0[3] = {0.f, 0.f, 0.f};
    if (cn > 0) {
#pragma unroll
      for (int k = 0; k < 3; k++) bp[k] = body_pos[3 * b + k];
#pragma unroll
      for (int k = 0; k < 4; k++) bq[k] = body_quat[4 * b + k];
    }
    // the first joint's local rotation depends on qpos alone: every lane
    // evaluates it (sincos, normalisation) once, off the level chain
    float ql0[4] = {1.f, 0.f, 0.f, 0.f};
    if (jn > 0) {
#pragma unroll
      for (int k = 0; k < 3; k++) { ax0[k] = IMG_F(jnt_axis)[3 * ja + k]; jp0[k] = IMG_F(jnt_pos)[3 * ja + k]; }
      if (jt0 == 3) {
        axis_angle(ql0, ax0, qpos[qa0] - qpos0[qa0]);
      } else if (jt0 == 1) {
        ql0[0] = qpos[qa0]; ql0[1] = qpos[qa0 + 1]; ql0[2] = qpos[qa0 + 2]; ql0[3] = qpos[qa0 + 3];
        quat_normalize(ql0);
      }
    }
    for (int lev = 1; __any(cn >= lev); lev++) {  // wave-uniform: up to the tree depth
      float pp[3], pq[4];
#pragma unroll
      for (int k = 0; k < 3; k++) pp[k] = shfl(p[k], par);
#pragma unroll
      for (int k = 0; k < 4; k++) pq[k] = shfl(q[k], par);
      if (cn != lev) continue;
      if (mid >= 0) {  // mocap body (a child of the world): pose from mocap_pos / mocap_quat
        const float* mp = DP(mocap_pos) + (W * Z.nmocap + mid) * 3;
        const float* mq = DP(mocap_quat) + (W * Z.nmocap + mid) * 4;
        p[0] = mp[0]; p[1] = mp[1]; p[2] = mp[2];
        q[0] = mq[0]; q[1] = mq[1]; q[2] = mq[2]; q[3] = mq[3];
        quat_normalize(q);
        continue;
      }
      if (jn == 1 && jt0 == 0) {  // free joint: the pose is the joint's coordinates
        p[0] = qpos[qa0]; p[1] = qpos[qa0 + 1]; p[2] = qpos[qa0 + 2];
        q[0] = qpos[qa0 + 3]; q[1] = qpos[qa0 + 4]; q[2] = qpos[qa0 + 5]; q[3] = qpos[qa0 + 6];
        quat_normalize(q);
        float R[9];
        quat2mat(R, q);
        xanchor[3 * ja] = p[0]; xanchor[3 * ja + 1] = p[1]; xanchor[3 * ja + 2] = p[2];
        xaxis[3 * ja] = R[2]; xaxis[3 * ja + 1] = R[5]; xaxis[3 * ja + 2] = R[8];
        continue;
      }
      {
        float R[9], t[3];
        quat2mat(R, pq);
        mat_vec(t, R, bp);
        p[0] = pp[0] + t[0]; p[1] = pp[1] + t[1]; p[2] = pp[2] + t[2];
        quat_mul(q, pq, bq);
      }
      for (int j = ja; j < ja + jn; j++) {
        const bool first = j == ja;
        float ja_ax[3], ja_pos[3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
          ja_ax[k] = first ? ax0[k] : IMG_F(jnt_axis)[3 * j + k];
          ja_pos[k] = first ? jp0[k] : IMG_F(jnt_pos)[3 * j + k];
        }
        const int jt = first ? jt0 : IMG_I(jnt_type)[j], qa = first ? qa0 : IMG_I(jnt_qposadr)[j];
        float Rq[9], ax[3], anc[3];
        quat2mat(Rq, q);
        mat_vec(ax, Rq, ja_ax);
        mat_vec(anc, Rq, ja_pos);
        anc[0] += p[0]; anc[1] += p[1]; anc[2] += p[2];
        if (jt == 2) {
          const float dd = qpos[qa] - qpos0[qa];
          p[0] += ax[0] * dd; p[1] += ax[1] * dd; p[2] += ax[2] * dd;
        } else if (jt == 3 || jt == 1) {  // hinge (axis-angle) / ball (the normalised qpos quaternion), about the anchor
          float ql[4] = {ql0[0], ql0[1], ql0[2], ql0[3]}, v[3];
          if (!first) {
            if (jt == 3) {
              axis_angle(ql, ja_ax, qpos[qa] - qpos0[qa]);
            } else {
              ql[0] = qpos[qa]; ql[1] = qpos[qa + 1]; ql[2] = qpos[qa + 2]; ql[3] = qpos[qa + 3];
              quat_normalize(ql);
            }
          }
          quat_mul(q, q, ql);
          quat2mat(Rq, q);
          mat_vec(v, Rq, ja_pos);
          p[0] = anc[0] - v[0]; p[1] = anc[1] - v[1]; p[2] = anc[2] - v[2];
        }
        xanchor[3 * j] = anc[0]; xanchor[3 * j + 1] = anc[1]; xanchor[3 * j + 2] = anc[2];
        xaxis[3 * j] = ax[0]; xaxis[3 * j + 1] = ax[1]; xaxis[3 * j + 2] = ax[2];
      }
      quat_normalize(q);
    }
#endif
    float R[9];
    quat2mat(R, q);
    xpos[3 * b] = p[0]; xpos[3 * b + 1] = p[1]; xpos[3 * b + 2] = p[2];
    xquat[4 * b] = q[0]; xquat[4 * b + 1] = q[1]; xquat[4 * b + 2] = q[2]; xquat[4 * b + 3] = q[3];
#pragma unroll
    for (int k = 0; k < 9; k++) xmat[9 * b + k] = R[k];
    float t[3], IR[9], IM[9];
    mat_vec(t, R, body_ipos + 3 * b);
    r_xipos[0] = p[0] + t[0]; r_xipos[1] = p[1] + t[1]; r_xipos[2] = p[2] + t[2];
    xipos[3 * b] = r_xipos[0]; xipos[3 * b + 1] = r_xipos[1]; xipos[3 * b + 2] = r_xipos[2];
    quat2mat(IR, body_iquat + 4 * b);
    mat_mul(IM, R, IR);
#pragma unroll
    for (int k = 0; k < 9; k++) ximat[9 * b + k] = r_ximat[k] = IM[k];
  }
  wsync();

  PROF(27);
  // geoms (all written out; collision geoms kept in LDS) and sites. The next
  // geom's inputs are loaded before this geom's stores (a load behind a store
  // waits for it).
  {
    int g = tid;
    float R[9], P[3];
    auto load_in = [&](int gg, float (&R_)[9], float (&P_)[3]) {
      const int b = IMG_I(geom_bodyid)[gg];
#pragma unroll
      for (int k = 0; k < 9; k++) R_[k] = xmat[9 * b + k];
#pragma unroll
      for (int k = 0; k < 3; k++) P_[k] = xpos[3 * b + k];
    };
    if (g < Z.ngeom) load_in(g, R, P);
    while (g < Z.ngeom) {
      float t[3], GR[9], GM[9];
      mat_vec(t, R, geom_pos + 3 * g);
      const float gp[3] = {P[0] + t[0], P[1] + t[1], P[2] + t[2]};
      quat2mat(GR, geom_quat + 4 * g);
      mat_mul(GM, R, GR);
      const int gn = g + NT;
      if (gn < Z.ngeom) load_in(gn, R, P);
      float* og = DP(geom_xpos) + W * Z.ngeom * 3 + 3 * g;
      og[0] = gp[0]; og[1] = gp[1]; og[2] = gp[2];
      float* om = DP(geom_xmat) + W * Z.ngeom * 9 + 9 * g;
#pragma unroll
      for (int k = 0; k < 9; k++) om[k] = GM[k];
      const int slot = IMG_I(geom_colslot)[g];
      if (slot >= 0) {
        cgpos[3 * slot] = gp[0]; cgpos[3 * slot + 1] = gp[1]; cgpos[3 * slot + 2] = gp[2];
#pragma unroll
        for (int k = 0; k < 9; k++) cgmat[9 * slot + k] = GM[k];
      }
      g = gn;
    }
  }
  PROF(28);
  for (int s = tid; s < Z.nsite; s += NT) {
    const int b = IMG_I(site_bodyid)[s];
    float R[9], P[3], t[3], SR[9], SM[9];
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = xmat[9 * b + k];
#pragma unroll
    for (int k = 0; k < 3; k++) P[k] = xpos[3 * b + k];
    mat_vec(t, R, site_pos + 3 * s);
    quat2mat(SR, site_quat + 4 * s);
    mat_mul(SM, R, SR);
    sxpos[3 * s] = P[0] + t[0]; sxpos[3 * s + 1] = P[1] + t[1]; sxpos[3 * s + 2] = P[2] + t[2];
#pragma unroll
    for (int k = 0; k < 9; k++) sxmat[9 * s + k] = SM[k];
  }

  // ---------------------------------------------------------------- com_pos
  PROF(1);
  // subtree com: lane b sums the bodies k whose chain contains b (ascending k)
  float r_sc[3];
  {
    const float bm = bl ? body_mass[tid] : 0.f;
    float ms = 0.f, mp0 = 0.f, mp1 = 0.f, mp2 = 0.f;
    for (int k = 0; k < nb; k++) {
      // masked accumulation as a multiply by 0/1 (no select per term): adds
      // exactly 0 for bodies outside the subtree
      const float mk = (tid == 0 || ((rl64(r_tmk, k) >> tid) & 1ull)) ? rl(bm, k) : 0.f;
      const float x0 = rl(r_xipos[0], k), x1 = rl(r_xipos[1], k), x2 = rl(r_xipos[2], k);
      ms += mk;
      mp0 += mk * x0; mp1 += mk * x1; mp2 += mk * x2;
    }
    if (ms < MJH_MINVAL) {
      r_sc[0] = r_xipos[0]; r_sc[1] = r_xipos[1]; r_sc[2] = r_xipos[2];
    } else {
      const float inv = 1.f / ms;
      r_sc[0] = mp0 * inv; r_sc[1] = mp1 * inv; r_sc[2] = mp2 * inv;
    }
    if (bl) { subtree_com[3 * tid] = r_sc[0]; subtree_com[3 * tid + 1] = r_sc[1]; subtree_com[3 * tid + 2] = r_sc[2]; }
  }
  // cinert (lane b), about the subtree com of b's root body
  {
    const int rt = bl ? IMG_I(body_rootid)[tid] : 0;
    const float c0 = shfl(r_sc[0], rt), c1 = shfl(r_sc[1], rt), c2 = shfl(r_sc[2], rt);
    const float* R = r_ximat;
    const float dd0 = r_xipos[0] - c0, dd1 = r_xipos[1] - c1, dd2 = r_xipos[2] - c2;
    const int bb = bl ? tid : 0;
    const float* in = body_inertia + 3 * bb;
    float I[6];  // xx yy zz xy xz yz of R diag(in) R^T
    I[0] = R[0] * in[0] * R[0] + R[1] * in[1] * R[1] + R[2] * in[2] * R[2];
    I[1] = R[3] * in[0] * R[3] + R[4] * in[1] * R[4] + R[5] * in[2] * R[5];
    I[2] = R[6] * in[0] * R[6] + R[7] * in[1] * R[7] + R[8] * in[2] * R[8];
    I[3] = R[0] * in[0] * R[3] + R[1] * in[1] * R[4] + R[2] * in[2] * R[5];
    I[4] = R[0] * in[0] * R[6] + R[1] * in[1] * R[7] + R[2] * in[2] * R[8];
    I[5] = R[3] * in[0] * R[6] + R[4] * in[1] * R[7] + R[5] * in[2] * R[8];
    const float mm = bl ? body_mass[bb] : 0.f, dsq = dd0 * dd0 + dd1 * dd1 + dd2 * dd2;
    r_cin[0] = I[0] + mm * (dsq - dd0 * dd0);
    r_cin[1] = I[1] + mm * (dsq - dd1 * dd1);
    r_cin[2] = I[2] + mm * (dsq - dd2 * dd2);
    r_cin[3] = I[3] - mm * dd0 * dd1;
    r_cin[4] = I[4] - mm * dd0 * dd2;
    r_cin[5] = I[5] - mm * dd1 * dd2;
    r_cin[6] = mm * dd0; r_cin[7] = mm * dd1; r_cin[8] = mm * dd2; r_cin[9] = mm;
    if (bl) {
#pragma unroll
      for (int c = 0; c < 10; c++) cinert[10 * tid + c] = r_cin[c];
    }
  }
  PROF(18);
  wsync();  // subtree_com visible to the per-joint lanes
#if MJH_CDOF_LANE
  // lane i = dof i builds its own cdof row (the per-joint rows below, row by
  // row: the same operations), kept in registers for the crb pass instead of
  // stored and reloaded through global scratch
  if (tid < nv) {
    const int i = tid;
    const int jn = IMG_I(dof_jntid)[i], b = IMG_I(dof_bodyid)[i];
    const int da = IMG_I(jnt_dofadr)[jn], t = IMG_I(jnt_type)[jn];
    const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
    const float off[3] = {c[0] - xanchor[3 * jn], c[1] - xanchor[3 * jn + 1], c[2] - xanchor[3 * jn + 2]};
    const int k = i - da;
    float row[6];
    if (t == 0 && k < 3) {  // free joint translation k
      row[0] = row[1] = row[2] = 0.f;
      row[3] = k == 0 ? 1.f : 0.f; row[4] = k == 1 ? 1.f : 0.f; row[5] = k == 2 ? 1.f : 0.f;
    } else if (t == 2) {  // slide
      row[0] = row[1] = row[2] = 0.f;
      row[3] = xaxis[3 * jn]; row[4] = xaxis[3 * jn + 1]; row[5] = xaxis[3 * jn + 2];
    } else {  // rotation: free joint rotation k-3 / ball k (the body's axes), hinge (its axis)
      float ax[3];
      if (t == 0 || t == 1) {
        const int kk = t == 0 ? k - 3 : k;
        ax[0] = xmat[9 * b + kk]; ax[1] = xmat[9 * b + 3 + kk]; ax[2] = xmat[9 * b + 6 + kk];
      } else {
        ax[0] = xaxis[3 * jn]; ax[1] = xaxis[3 * jn + 1]; ax[2] = xaxis[3 * jn + 2];
      }
      row[0] = ax[0]; row[1] = ax[1]; row[2] = ax[2];
      cross3(&row[3], ax, off);
    }
#pragma unroll
    for (int e = 0; e < 6; e++) {
      cdof[6 * i + e] = row[e];
      r_cdof[e] = row[e];
    }
  }
  if (false)
#endif
  for (int j = tid; j < nj; j += NT) {
    // every input is loaded before the first cdof store (a load behind a store
    // waits for it)
    const int b = IMG_I(jnt_bodyid)[j], da = IMG_I(jnt_dofadr)[j];
    const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
    float off[3] = {c[0] - xanchor[3 * j], c[1] - xanchor[3 * j + 1], c[2] - xanchor[3 * j + 2]};
    const int t = IMG_I(jnt_type)[j];
    if (t == 0) {
      float R[9];
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = xmat[9 * b + k];
      float rows[6][6];
#pragma unroll
      for (int k = 0; k < 3; k++) {
#pragma unroll
        for (int e = 0; e < 6; e++) rows[k][e] = e == 3 + k ? 1.f : 0.f;
        const float ax[3] = {R[k], R[3 + k], R[6 + k]};
        rows[3 + k][0] = ax[0]; rows[3 + k][1] = ax[1]; rows[3 + k][2] = ax[2];
        cross3(&rows[3 + k][3], ax, off);
      }
#pragma unroll
      for (int k = 0; k < 6; k++)
#pragma unroll
        for (int e = 0; e < 6; e++) cdof[6 * (da + k) + e] = rows[k][e];
    } else if (t == 1) {  // ball: rotations about the body's axes
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const float ax[3] = {xmat[9 * b + k], xmat[9 * b + 3 + k], xmat[9 * b + 6 + k]};
        float cr[3];
        cross3(cr, ax, off);
        float* cd = cdof + 6 * (da + k);
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cd[3] = cr[0]; cd[4] = cr[1]; cd[5] = cr[2];
      }
    } else {
      const float ax[3] = {xaxis[3 * j], xaxis[3 * j + 1], xaxis[3 * j + 2]};
      float* cd = cdof + 6 * da;
      if (t == 2) {
        cd[0] = cd[1] = cd[2] = 0.f;
        cd[3] = ax[0]; cd[4] = ax[1]; cd[5] = ax[2];
      } else {
        float cr[3];
        cross3(cr, ax, off);
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cd[3] = cr[0]; cd[4] = cr[1]; cd[5] = cr[2];
      }
    }
  }
  wsync();

  PROF(19);
  // ---------------------------------------------------------------- crb + M
  // lane i's cdof row in registers
  if (!MJH_CDOF_LANE && tid < nv) {
#pragma unroll
    for (int c = 0; c < 6; c++) r_cdof[c] = cdof[6 * tid + c];
  }
  // crb (lane b) = sum of cinert over b's subtree, ascending k
  float r_crb[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // not unrolled: a fully unrolled body loop hoists every readlane and spills
  // the scalar results into VGPR lanes
#pragma nounroll
  for (int k = 1; k < nb; k++) {
    const float in = (tid > 0 && ((rl64(r_tmk, k) >> tid) & 1ull)) ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < 10; c++) r_crb[c] = fmaf(rl(r_cin[c], k), in, r_crb[c]);  // exact: x*1 + r, or r + 0
  }
  PROF(20);
  {
    // lane i builds row i of M in registers: the entries j <= i over i's
    // ancestor chain (cdof_j . crb_b(i) cdof_i), then the entries j > i from the
    // rows the other lanes stored (M is symmetric). Whole-row stores only (no
    // zero fill, no column scatter), and the factorisation starts from the
    // registers. Rows of lanes >= nv are inert identity rows (never stored).
    const int bi = tid < nv ? IMG_I(dof_bodyid)[tid] : 0;
    float cb[10], buf[6];
#pragma unroll
    for (int c = 0; c < 10; c++) cb[c] = shfl(r_crb[c], bi);
    inert_vec(buf, cb, r_cdof);
    unsigned long long mask = tid < nv ? dmk[bi] : 0ull;
    mask &= (tid == 63) ? ~0ull : ((2ull << tid) - 1ull);
    const float arm = tid < nv ? dof_armature[tid] : 0.f;
    float a[NVP];
#pragma unroll
    for (int j = 0; j < NVP; j++) {
      float cj[6];
#pragma unroll
      for (int c = 0; c < 6; c++) cj[c] = rl(r_cdof[c], j);
      float v = cj[0] * buf[0] + cj[1] * buf[1] + cj[2] * buf[2] + cj[3] * buf[3] + cj[4] * buf[4] + cj[5] * buf[5];
      if (j == tid) v += arm;
      a[j] = ((mask >> j) & 1ull) ? v : 0.f;
    }
    if (tid < nv) {
      float* r = Lm + lofs<PKL>(tid, ldm);
      const int len = lspan<PKL>(tid, ldm);
#pragma unroll
      for (int k = 0; k < NVP; k += 4)
        if (k < len) *reinterpret_cast<float4*>(r + k) = make_float4(a[k], a[k + 1], a[k + 2], a[k + 3]);
    }
    wsync();
    if (tid < nv) {
#pragma unroll
      for (int j = 1; j < NVP; j++)
        if (j > tid && j < nv) a[j] = Lm[lofs<PKL>(j, ldm) + tid];
      float* r = Mm + tid * ldm;
#pragma unroll
      for (int k = 0; k < NVP; k += 4) *reinterpret_cast<float4*>(r + k) = make_float4(a[k], a[k + 1], a[k + 2], a[k + 3]);
    } else {
#pragma unroll
      for (int j = 0; j < NVP; j++) a[j] = j == tid ? 1.f : 0.f;
    }
    PROF(10);
    ldl_factor_rows<NVP, PKL>(a, Lm, nv, ldm);
  }
  PROF(2);

  // ---------------------------------------------------------------- collision
  {
    const int npair = Z.npair;
    for (int base = 0; base < npair; base += NT) {
      const int p = base + tid;
      Con cc[4];
      int n = 0, g1 = 0, g2 = 0;
      if (p < npair) {
#if MJH_PAIR_REC
        const int4* rec = reinterpret_cast<const int4*>(IMGB + Io.pair_rec) + 2 * p;
        const int4 ra = rec[0], rb = rec[1];
        g1 = ra.x;
        g2 = ra.y;
        const int s1 = ra.z, s2 = ra.w, t1 = rb.x, t2 = rb.y;
        const float margin = __int_as_float(rb.z), reach = __int_as_float(rb.w);
#else
        g1 = IMG_I(pair_geom1)[p];
        g2 = IMG_I(pair_geom2)[p];
        const int s1 = IMG_I(geom_colslot)[g1], s2 = IMG_I(geom_colslot)[g2];
        const float margin = fmaxf(IMG_F(geom_margin)[g1], IMG_F(geom_margin)[g2]);
        const int t1 = IMG_I(geom_type)[g1], t2 = IMG_I(geom_type)[g2];
        const float reach = t1 == 0 ? margin + IMG_F(geom_rbound)[g2] : margin + IMG_F(geom_rbound)[g1] + IMG_F(geom_rbound)[g2];
#endif
        const float* p1 = cgpos + 3 * s1;
        const float* p2 = cgpos + 3 * s2;
        const float* m1 = cgmat + 9 * s1;
        const float* m2 = cgmat + 9 * s2;
        float dif[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
        bool near;
        if (t1 == 0) {
          float nrm[3] = {m1[2], m1[5], m1[8]};
          near = dot3(dif, nrm) <= reach;
        } else {
          near = sqrtf(dot3(dif, dif)) <= reach;
        }
        if (near)
          n = narrowphase(t1, t2, p1, m1, IMG_F(geom_size) + 3 * g1, p2, m2, IMG_F(geom_size) + 3 * g2, margin, cc,
                          Z.nboxpair > 0);
      }
      int total;
      const int off = bscan<NT>(n, &total, redi);
      const int base_con = ints[I_NCON];
      if (n > 0) {
        // contact parameters (mj_contactParam semantics)
        int condim;
        float fri[3], solref[2], solimp[5];
        const int pr1 = IMG_I(geom_priority)[g1], pr2 = IMG_I(geom_priority)[g2];
        if (pr1 != pr2) {
          const int g = pr1 > pr2 ? g1 : g2;
          condim = IMG_I(geom_condim)[g];
          for (int k = 0; k < 3; k++) fri[k] = geom_friction[3 * g + k];
          for (int k = 0; k < 2; k++) solref[k] = IMG_F(geom_solref)[2 * g + k];
          for (int k = 0; k < 5; k++) solimp[k] = IMG_F(geom_solimp)[5 * g + k];
        } else {
          condim = max(IMG_I(geom_condim)[g1], IMG_I(geom_condim)[g2]);
          for (int k = 0; k < 3; k++) fri[k] = fmaxf(geom_friction[3 * g1 + k], geom_friction[3 * g2 + k]);
          const float sm1 = IMG_F(geom_solmix)[g1], sm2 = IMG_F(geom_solmix)[g2];
          float mix;
          if (sm1 >= MJH_MINVAL && sm2 >= MJH_MINVAL) mix = sm1 / (sm1 + sm2);
          else if (sm1 < MJH_MINVAL && sm2 < MJH_MINVAL) mix = 0.5f;
          else mix = sm1 < MJH_MINVAL ? 0.f : 1.f;
          const float* r1 = IMG_F(geom_solref) + 2 * g1;
          const float* r2 = IMG_F(geom_solref) + 2 * g2;
          if (r1[0] > 0.f && r2[0] > 0.f)
            for (int k = 0; k < 2; k++) solref[k] = mix * r1[k] + (1.f - mix) * r2[k];
          else
            for (int k = 0; k < 2; k++) solref[k] = fminf(r1[k], r2[k]);
          for (int k = 0; k < 5; k++) solimp[k] = mix * IMG_F(geom_solimp)[5 * g1 + k] + (1.f - mix) * IMG_F(geom_solimp)[5 * g2 + k];
        }
        const float imargin = fmaxf(IMG_F(geom_margin)[g1], IMG_F(geom_margin)[g2]) - fmaxf(IMG_F(geom_gap)[g1], IMG_F(geom_gap)[g2]);
        for (int e = 0; e < n; e++) {
          const int ci = base_con + off + e;
          if (ci >= Lo.ncap) {
            ints[I_FLAGS] |= MJH_FLAG_CONTACT_OVERFLOW;  // benign race: all writers set the same bit
            break;
          }
          float fr[9] = {cc[e].frame[0], cc[e].frame[1], cc[e].frame[2], cc[e].frame[3], cc[e].frame[4], cc[e].frame[5], 0.f, 0.f, 0.f};
          make_frame(fr);
          con_dist[ci] = cc[e].dist;
          for (int k = 0; k < 3; k++) con_pos[3 * ci + k] = cc[e].pos[k];
          for (int k = 0; k < 9; k++) con_frame[9 * ci + k] = fr[k];
          con_fric[5 * ci] = fri[0]; con_fric[5 * ci + 1] = fri[0]; con_fric[5 * ci + 2] = fri[1];
          con_fric[5 * ci + 3] = fri[2]; con_fric[5 * ci + 4] = fri[2];
          con_solref[2 * ci] = solref[0]; con_solref[2 * ci + 1] = solref[1];
          for (int k = 0; k < 5; k++) con_solimp[5 * ci + k] = solimp[k];
          con_imargin[ci] = imargin;
          con_dim[ci] = condim;
          con_geom[2 * ci] = g1;
          con_geom[2 * ci + 1] = g2;
          con_efcadr[ci] = -1;
        }
      }
      wsync();
      if (tid == 0) ints[I_NCON] = min(base_con + total, Lo.ncap);
      wsync();
    }
  }
  ncon = ints[I_NCON];
  PROF(4);
  }  // position stage, part 1 (kinematics .. collision)

  // ---------------------------------------------------------------- row capacity
  // The constraint rows' arrays live in LDS for up to Lo.lcap rows. A world with
  // more rows (one-world workgroups, lcap < rcap = njmax) runs the rest of the
  // step with them in global scratch instead (BIG): the same code on other
  // addresses, so its results are the same. Its row count is known before any
  // row is written: the counts of the rows make_constraint emits (frictionloss
  // dofs, active limits, contacts within their margin) or the handoff's.
  constexpr bool kTwoTier = cu_worlds(WPB) && MODE != 1;
  bool big = false;
  if constexpr (kTwoTier) {
    if (Lo.lcap < Lo.rcap) {
      int need = 0;
      if (MODE == 2 || reused) {
        need = reinterpret_cast<const int*>(G + Lo.h_ints)[I_NEFC];
      } else {
        for (int base = 0; base < nv; base += NT) {
          const int i = base + tid;
          need += __popcll(__ballot(i < nv && dof_frictionloss[i] > 0.f));
        }
        for (int base = 0; base < nj; base += NT) {
          const int j = base + tid;
          bool f = false;
          if (j < nj && IMG_I(jnt_limited)[j]) {
            float pos, sgn;
            f = joint_limit(IMG_I(jnt_type)[j], qpos + IMG_I(jnt_qposadr)[j], jnt_range + 2 * j, IMG_F(jnt_margin)[j],
                            &pos, &sgn);
          }
          need += __popcll(__ballot(f));
        }
        for (int base = 0; base < ncon; base += NT) {
          const int ci = base + tid;
          int nr = 0;
          if (ci < ncon && con_dist[ci] - con_imargin[ci] < 0.f)
            nr = con_dim[ci] == 1 ? 1 : (ELL ? con_dim[ci] : 2 * (con_dim[ci] - 1));
          int total;
          (void)bscan<NT>(nr, &total, redi);
          need += total;
        }
      }
      big = need > Lo.lcap;
    }
  }

  auto tail = [&](auto big_tag) {
  constexpr bool BIG = decltype(big_tag)::value;
  // row arrays: LDS (or the preset's region) for up to lcap rows, global scratch for BIG worlds
#define SPR(name) (BIG && !Rg::name ? G + Lo.g_##name : SP(name))
#define SPRI(name) reinterpret_cast<int*>(SPR(name))
  float* efc_D = HO ? G + Lo.h_D : SPR(efc_D);
  float* efc_R = HO ? G + Lo.h_R : SPR(efc_R);
  float* efc_aref = HO ? G + Lo.h_aref : SPR(efc_aref);
  float* jaref = SPR(efc_jaref);
  float* jv = HO ? G + Lo.h_jv : SPR(efc_jv);
  float* efc_force = SPR(efc_force);
  float* efc_fl = HO ? G + Lo.h_fl : SPR(efc_fl);
  int* efc_type = HO ? reinterpret_cast<int*>(G + Lo.h_type) : SPRI(efc_type);
  float* efc_h = SPR(efc_h);
  int* arow = SPRI(arow);
  float* ash = SPR(ash);
  // the damping coefficient of each row until the velocity stage completes aref
  float* efc_b = MODE == 0 ? SPR(efc_h) : G + Lo.h_b;
#undef SPRI
#undef SPR
  const int acap = (BIG || Rg::arow) ? Lo.rcap : Lo.lcap;  // arow's entries
  const int tcap = (BIG || Rg::efc_type) ? Lo.rcap : Lo.lcap;  // the row arrays' entries (efc_type's region)
  if (MODE == 1 || (MODE == 0 && !reused)) {  // position stage, part 2

  // ---------------------------------------------------------------- make_constraint
  {
    int nefc = 0;
    const int rcap = Lo.rcap;
    // dof friction loss rows
    for (int base = 0; base < nv; base += NT) {
      const int i = base + tid;
      const int f = (i < nv && dof_frictionloss[i] > 0.f) ? 1 : 0;
      int total;
      const int off = bscan<NT>(f, &total, redi);
      if (f) {
        const int r = nefc + off;
        if (r < rcap && MJH_BOK(r, tcap)) {
          efc_type[r] = MJH_CNSTR_FRICTION_DOF;
          efc_id[r] = i;
          efc_fl[r] = dof_frictionloss[i];
          efc_mask[r] = 1ull << i;
          efc_pos[r] = 0.f;
          row_params_pos(m.timestep, 0.f, 0.f, IMG_F(dof_invweight0)[i], IMG_F(dof_solref) + 2 * i,
                         IMG_F(dof_solimp) + 5 * i, efc_D + r, efc_R + r, efc_aref + r, efc_b + r);
        }
      }
      nefc += total;
    }
    // joint limits
    for (int base = 0; base < nj; base += NT) {
      const int j = base + tid;
      int f = 0;
      float pos = 0.f, sgn = 0.f;
      if (j < nj && IMG_I(jnt_limited)[j])
        f = joint_limit(IMG_I(jnt_type)[j], qpos + IMG_I(jnt_qposadr)[j], jnt_range + 2 * j, IMG_F(jnt_margin)[j], &pos,
                        &sgn) ? 1 : 0;
      int total;
      const int off = bscan<NT>(f, &total, redi);
      if (f) {
        const int r = nefc + off;
        if (r < rcap && MJH_BOK(r, tcap)) {
          const int dof = IMG_I(jnt_dofadr)[j];
          efc_type[r] = MJH_CNSTR_LIMIT_JOINT;
          efc_id[r] = j;
          efc_fl[r] = 0.f;
          efc_mask[r] = (IMG_I(jnt_type)[j] == 1 ? 7ull : 1ull) << dof;  // a ball limit spans its three dofs
          efc_pos[r] = pos + IMG_F(jnt_margin)[j];
          jv[r] = sgn;  // temporarily hold the Jacobian sign
          row_params_pos(m.timestep, pos, pos, IMG_F(dof_invweight0)[dof], IMG_F(jnt_solref) + 2 * j,
                         IMG_F(jnt_solimp) + 5 * j, efc_D + r, efc_R + r, efc_aref + r, efc_b + r);
        }
      }
      nefc += total;
    }
    const int nsimple = min(nefc, rcap);
    // contact rows
    for (int base = 0; base < ncon; base += NT) {
      const int ci = base + tid;
      int nr = 0;
      if (ci < ncon && con_dist[ci] - con_imargin[ci] < 0.f)
        nr = con_dim[ci] == 1 ? 1 : (ELL ? con_dim[ci] : 2 * (con_dim[ci] - 1));
      int total;
      const int off = bscan<NT>(nr, &total, redi);
      if (nr) {
        const int r0 = nefc + off;
        if (r0 + nr <= rcap) {
          con_efcadr[ci] = r0;
        } else {
          con_efcadr[ci] = -1;
          atomicMin(&ints[I_MISC], r0);  // rows of this and later contacts are dropped
        }
      }
      nefc += total;
    }
    wsync();
    if (nefc > rcap) {
      if (tid == 0) ints[I_FLAGS] |= MJH_FLAG_EFC_OVERFLOW;
      nefc = max(nsimple, min(rcap, ints[I_MISC]));
    }
    wsync();
    // J rows with lane = column: every entry of every row is stored (zeros
    // included, so no zero fill) as coalesced row stores, and all of a round's
    // inputs are loaded before its first store (a load behind a store waits for
    // it). Single-dof rows first, their (type, column, value) one per lane.
    for (int base = 0; base < nsimple; base += NT) {
      int col = -1;
      float val = 0.f, bv[3] = {0.f, 0.f, 0.f};
      bool ball = false;
      if (base + tid < nsimple) {
        const int r = base + tid, t = efc_type[r];
        col = t == MJH_CNSTR_FRICTION_DOF ? efc_id[r] : IMG_I(jnt_dofadr)[efc_id[r]];
        val = t == MJH_CNSTR_FRICTION_DOF ? 1.f : jv[r];
        if (t == MJH_CNSTR_LIMIT_JOINT && IMG_I(jnt_type)[efc_id[r]] == 1) {
          // ball limit: -(unit rotation axis) on the joint's three dofs
          ball = true;
          quat2vel(bv, qpos + IMG_I(jnt_qposadr)[efc_id[r]]);
          normalize3(bv);
          val = -bv[0];
        }
      }
      const int cnt = min(NT, nsimple - base);
      if (__ballot(ball) == 0ull) {
        for (int k = 0; k < cnt; k++) {
          const int ck = __builtin_amdgcn_readlane(col, k);
          const float vk = rl(val, k);
          if (tid < ldj) J[(base + k) * ldj + tid] = tid == ck ? vk : 0.f;
        }
      } else {  // rows with up to three consecutive entries
        const float b1 = ball ? -bv[1] : 0.f, b2 = ball ? -bv[2] : 0.f;
        for (int k = 0; k < cnt; k++) {
          const int ck = __builtin_amdgcn_readlane(col, k);
          const float vk = rl(val, k), v1 = rl(b1, k), v2 = rl(b2, k);
          if (tid < ldj) J[(base + k) * ldj + tid] = tid == ck ? vk : (tid == ck + 1 ? v1 : (tid == ck + 2 ? v2 : 0.f));
        }
      }
    }
    // contact rows: lane = contact loads the contact's data, then per contact
    // (uniform) lane = dof builds the rows' column entries
    {
      float cd[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (tid < nv) {
#pragma unroll
        for (int c = 0; c < 6; c++) cd[c] = cdof[6 * tid + c];
      }
      for (int base = 0; base < ncon; base += NT) {
        const int cl = base + tid;
        int r0 = -1, b1 = 0, b2 = 0, dim = 1;
        unsigned long long m1 = 0ull, m2 = 0ull;  // the bodies' dof masks (no image load in the row loop below)
        float cp[3] = {0.f, 0.f, 0.f}, fr[9], fk[5], c1[3] = {0.f, 0.f, 0.f}, c2[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 9; k++) fr[k] = 0.f;
#pragma unroll
        for (int k = 0; k < 5; k++) fk[k] = 0.f;
        if (cl < ncon) {
          r0 = con_efcadr[cl];
          b1 = IMG_I(geom_bodyid)[con_geom[2 * cl]];
          b2 = IMG_I(geom_bodyid)[con_geom[2 * cl + 1]];
          dim = con_dim[cl];
          m1 = IMG_L(body_dofmask)[b1];
          m2 = IMG_L(body_dofmask)[b2];
#pragma unroll
          for (int k = 0; k < 3; k++) cp[k] = con_pos[3 * cl + k];
#pragma unroll
          for (int k = 0; k < 9; k++) fr[k] = con_frame[9 * cl + k];
#pragma unroll
          for (int k = 0; k < 5; k++) fk[k] = con_fric[5 * cl + k];
          const float* s1 = subtree_com + 3 * IMG_I(body_rootid)[b1];
          const float* s2 = subtree_com + 3 * IMG_I(body_rootid)[b2];
#pragma unroll
          for (int k = 0; k < 3; k++) { c1[k] = s1[k]; c2[k] = s2[k]; }
        }
        const int cnt = min(NT, ncon - base);
        for (int k = 0; k < cnt; k++) {
          const int r0k = __builtin_amdgcn_readlane(r0, k);
          if (r0k < 0) continue;
          const unsigned long long m1k = rl64(m1, k), m2k = rl64(m2, k);
          const int dimk = __builtin_amdgcn_readlane(dim, k);
          const int nr = dimk == 1 ? 1 : 2 * (dimk - 1);  // pyramidal (elliptic: dimk rows)
          const bool in1 = tid < nv && ((m1k >> tid) & 1ull);
          const bool in2 = tid < nv && ((m2k >> tid) & 1ull);
          // not in either chain, or in both (relative motion cancels): zero column
          const bool use = in1 != in2;
          const float sg = in2 ? 1.f : -1.f;
          float off[3], t[3];
#pragma unroll
          for (int q = 0; q < 3; q++) off[q] = rl(cp[q], k) - (in2 ? rl(c2[q], k) : rl(c1[q], k));
          cross3(t, cd, off);
          const float jp[3] = {sg * (cd[3] + t[0]), sg * (cd[4] + t[1]), sg * (cd[5] + t[2])};
          const float jr[3] = {sg * cd[0], sg * cd[1], sg * cd[2]};
          float f[9];
#pragma unroll
          for (int q = 0; q < 9; q++) f[q] = rl(fr[q], k);
          float jf[6];
          jf[0] = dot3(f, jp); jf[1] = dot3(f + 3, jp); jf[2] = dot3(f + 6, jp);
          jf[3] = dot3(f, jr); jf[4] = dot3(f + 3, jr); jf[5] = dot3(f + 6, jr);
          if (tid < ldj) {
            if (dimk == 1) {
              J[r0k * ldj + tid] = use ? jf[0] : 0.f;
            } else if (ELL) {
              // elliptic: row e is the frame component e (translational for
              // e < 3, rotational after)
#pragma unroll
              for (int e = 0; e < 6; e++)
                if (e < dimk) J[(r0k + e) * ldj + tid] = use ? jf[e] : 0.f;
            } else {
              float fkv[5];
#pragma unroll
              for (int q = 0; q < 5; q++) fkv[q] = rl(fk[q], k);
              // pyramid edges e = 2(kk-1), 2(kk-1)+1 of friction direction kk
              // (static register indices: no private-memory arrays)
#pragma unroll
              for (int kk = 1; kk < 6; kk++) {
                if (2 * (kk - 1) >= nr) break;
                const int e = 2 * (kk - 1);
                J[(r0k + e) * ldj + tid] = use ? jf[0] + fkv[kk - 1] * jf[kk] : 0.f;
                J[(r0k + e + 1) * ldj + tid] = use ? jf[0] + (-fkv[kk - 1]) * jf[kk] : 0.f;
              }
            }
          }
        }
      }
    }
    // contact rows' type, mask and parameters: lane = contact, every input loaded
    // before the first row store (a load behind a store waits for it). The rows of
    // a frictionless or pyramidal contact share one set of parameters (MuJoCo
    // Warp's per-row evaluation computes the same values from the same inputs).
    for (int ci = tid; ci < ncon; ci += NT) {
      const int r0 = con_efcadr[ci];
      if (r0 < 0) continue;
      const int b1 = IMG_I(geom_bodyid)[con_geom[2 * ci]], b2 = IMG_I(geom_bodyid)[con_geom[2 * ci + 1]];
      const int dim = con_dim[ci];
      const bool ell = ELL && dim > 1;
      const int nr = dim == 1 ? 1 : (ell ? dim : 2 * (dim - 1));
      const unsigned long long msk =
          (unsigned long long)IMG_L(body_dofmask)[b1] ^ (unsigned long long)IMG_L(body_dofmask)[b2];
      const float dist = con_dist[ci], imarg = con_imargin[ci], f0 = con_fric[5 * ci];
      const float pos = dist - imarg;
      const float invw0 = IMG_F(body_invweight0)[2 * b1] + IMG_F(body_invweight0)[2 * b2];
      float pD = 0.f, pR = 0.f, paref = 0.f, pb = 0.f;
      if (!ell) {
        float invw = invw0;
        if (dim > 1) {
          invw = invw + f0 * f0 * invw;
          invw = invw * 2.f * f0 * f0 / m.impratio;
        }
        row_params_pos(m.timestep, pos, pos, invw, con_solref + 2 * ci, con_solimp + 5 * ci, &pD, &pR, &paref, &pb);
      }
      for (int e = 0; e < nr; e++) {
        const int r = r0 + e;
        if (!MJH_BOK(r, tcap)) break;
        efc_type[r] = dim == 1 ? MJH_CNSTR_CONTACT_FRICTIONLESS
                               : (ell ? MJH_CNSTR_CONTACT_ELLIPTIC : MJH_CNSTR_CONTACT_PYRAMIDAL);
        efc_id[r] = ci;
        efc_mask[r] = msk;
        if (!ell) {
          efc_fl[r] = 0.f;
          efc_pos[r] = dist;
          efc_D[r] = pD; efc_R[r] = pR; efc_aref[r] = paref; efc_b[r] = pb;
          continue;
        }
        // elliptic: the cone's row scales (mu = friction0 / sqrt(impratio), then
        // friction_{e-1}); friction rows have no position term (efc_pos = margin,
        // as MuJoCo Warp), invweight / impratio, times f0^2 / f_{e-1}^2 beyond the
        // first (constraint.py _efc_contact_elliptic)
        const float fe = e > 0 ? con_fric[5 * ci + e - 1] : f0;
        efc_fl[r] = e == 0 ? f0 / sqrtf(m.impratio) : fe;
        efc_pos[r] = e > 0 ? imarg : dist;
        float invw = invw0;
        if (e > 0) {
          invw = invw / m.impratio;
          if (e > 1) invw *= f0 * f0 / (fe * fe);
        }
        row_params_pos(m.timestep, e > 0 ? 0.f : pos, pos, invw, con_solref + 2 * ci, con_solimp + 5 * ci, efc_D + r,
                       efc_R + r, efc_aref + r, efc_b + r);
      }
    }
    if (tid == 0) ints[I_NEFC] = nefc;
    wsync();
  }
  nefc = ints[I_NEFC];
  PROF(5);
  if (MODE == 0 && !STEP && reuse) {
    // a forward saves its position stage's LDS results (the factor of M, the
    // rows' position parameters, counters) and the snapshot: the next step
    // launch on an unchanged world (qpos is only integrated by steps, so the
    // first step after a forward) skips the position stage
    img_hash = image_hash();
    wsync();
    if (tid < I_COUNT) reinterpret_cast<int*>(G + Lo.h_ints)[tid] = ints[tid];
    for (int i = tid; i < kLWords; i += NT) G[Lo.h_L + i] = Lm[i];
    int* ht = reinterpret_cast<int*>(G + Lo.h_type);
    for (int r = tid; r < nefc; r += NT) {
      ht[r] = efc_type[r];
      G[Lo.h_fl + r] = efc_fl[r];
      G[Lo.h_D + r] = efc_D[r];
      G[Lo.h_R + r] = efc_R[r];
      G[Lo.h_aref + r] = efc_aref[r];
      G[Lo.h_b + r] = efc_b[r];
    }
    const unsigned* qb = reinterpret_cast<const unsigned*>(qpos);
    for (int i = tid; i < nq; i += NT) snap[7 + i] = qb[i];
    if (Z.nmocap > 0) {
      const unsigned* mp = reinterpret_cast<const unsigned*>(DP(mocap_pos) + W * Z.nmocap * 3);
      const unsigned* mq = reinterpret_cast<const unsigned*>(DP(mocap_quat) + W * Z.nmocap * 4);
      for (int i = tid; i < 3 * Z.nmocap; i += NT) snap[7 + nq + i] = mp[i];
      for (int i = tid; i < 4 * Z.nmocap; i += NT) snap[7 + nq + 3 * Z.nmocap + i] = mq[i];
    }
    if (tid == 0) {
      snap[1] = (unsigned)img_hash; snap[2] = (unsigned)(img_hash >> 32);
      snap[3] = (unsigned)wf_hash; snap[4] = (unsigned)(wf_hash >> 32);
      snap[5] = (unsigned)key; snap[6] = (unsigned)(key >> 32);
    }
    wsync();
    if (tid == 0) snap[0] = 1u;
  }
  }  // position stage
  if constexpr (MODE == 1) {
    // handoff: counters / overflow flags, then the snapshot that lets the next
    // pass skip this world while nothing it depends on changed
    wsync();
    if (tid < I_COUNT) reinterpret_cast<int*>(G + Lo.h_ints)[tid] = ints[tid];
    const unsigned* qb = reinterpret_cast<const unsigned*>(qpos);
    for (int i = tid; i < nq; i += NT) snap[7 + i] = qb[i];
    if (Z.nmocap > 0) {
      const unsigned* mp = reinterpret_cast<const unsigned*>(DP(mocap_pos) + W * Z.nmocap * 3);
      const unsigned* mq = reinterpret_cast<const unsigned*>(DP(mocap_quat) + W * Z.nmocap * 4);
      for (int i = tid; i < 3 * Z.nmocap; i += NT) snap[7 + nq + i] = mp[i];
      for (int i = tid; i < 4 * Z.nmocap; i += NT) snap[7 + nq + 3 * Z.nmocap + i] = mq[i];
    }
    if (tid == 0) {
      snap[1] = (unsigned)img_hash; snap[2] = (unsigned)(img_hash >> 32);
      snap[3] = (unsigned)wf_hash; snap[4] = (unsigned)(wf_hash >> 32);
      snap[5] = (unsigned)key; snap[6] = (unsigned)(key >> 32);
    }
    wsync();
    if (tid == 0) snap[0] = 1u;
    return;
  } else {
  if (MODE == 2 || reused) {
    // the position stage's results: counters, the rows' position parameters
    // (LDS for the solver), registers of the tree passes
    const int* ih = reinterpret_cast<const int*>(G + Lo.h_ints);
    if (tid < I_COUNT) ints[tid] = ih[tid];
    if (bl) {
#pragma unroll
      for (int c = 0; c < 10; c++) r_cin[c] = cinert[10 * tid + c];
    }
    if (tid < nv) {
#pragma unroll
      for (int c = 0; c < 6; c++) r_cdof[c] = cdof[6 * tid + c];
    }
    wsync();
    ncon = ints[I_NCON];
    nefc = ints[I_NEFC];
    const int* ht = reinterpret_cast<const int*>(G + Lo.h_type);
    for (int r = tid; r < nefc; r += NT) {
      efc_type[r] = ht[r];
      efc_fl[r] = G[Lo.h_fl + r];
      efc_D[r] = G[Lo.h_D + r];
      efc_R[r] = G[Lo.h_R + r];
      efc_aref[r] = G[Lo.h_aref + r];
      if constexpr (MODE == 0) efc_b[r] = G[Lo.h_b + r];
    }
    // the fused kernel keeps the factor of M in LDS
    if constexpr (MODE == 0)
      for (int i = tid; i < kLWords; i += NT) Lm[i] = G[Lo.h_L + i];
  }
  wsync();
  // aref = aref_pos - b J qvel (row_params: the velocity term)
  for (int r = tid; r < nefc; r += NT) {
    const float jq = rowdot_u<NVP>(J + r * ldj, qvel, nv);
    efc_aref[r] = efc_aref[r] - efc_b[r] * jq;
  }
  wsync();

  // ---------------------------------------------------------------- com_vel / rne (bias)
  const float r_qv = tid < nv ? qvel[tid] : 0.f;
  const unsigned long long r_dm = bl ? dmk[tid] : 0ull;
  float r_cvel[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nv; j++) {
    const float q = ((r_dm >> j) & 1ull) ? rl(r_qv, j) : 0.f;  // 0 outside the chain: adds exactly 0
#pragma unroll
    for (int c = 0; c < 6; c++) r_cvel[c] += rl(r_cdof[c], j) * q;
  }
  if (bl) {
#pragma unroll
    for (int c = 0; c < 6; c++) cvel[6 * tid + c] = r_cvel[c];
  }
  PROF(21);
  // cdof_dot (lane i)
  float r_cdd[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  {
    const int i = tid < nv ? tid : 0;
    const int b = IMG_I(dof_bodyid)[i], jnt = IMG_I(dof_jntid)[i], da = IMG_I(jnt_dofadr)[jnt];
    const bool freej = IMG_I(jnt_type)[jnt] == 0;
    const int p = IMG_I(body_parentid)[b], d0 = IMG_I(body_dofadr)[b];
    float v[6];
#pragma unroll
    for (int c = 0; c < 6; c++) v[c] = shfl(r_cvel[c], p);
    // earlier dofs of this body: other joints fully, own free joint translations
    // only. Only bodies with several dofs have any, so the loop ends at the
    // wave's largest such dof (G1/Go1: the free joint's, k < 5)
    int kend = (tid < nv && d0 < i) ? i : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) kend = max(kend, __shfl_xor(kend, o, 64));
    for (int k = 0; k < kend; k++) {
      const int jk = __builtin_amdgcn_readlane(jnt, k);  // dof k's joint (lane k < nv loaded it)
      const bool use = k >= d0 && k < i && !(jk == jnt && !(freej && k - da < 3));
      const float q = use ? rl(r_qv, k) : 0.f;  // adds exactly 0 when unused
#pragma unroll
      for (int c = 0; c < 6; c++) v[c] += rl(r_cdof[c], k) * q;
    }
    if (tid < nv && !(freej && i - da < 3)) cross_motion(r_cdd, v, r_cdof);
    if (tid < nv) {
#pragma unroll
      for (int c = 0; c < 6; c++) cdof_dot[6 * tid + c] = r_cdd[c];
    }
  }
  PROF(22);
  // rne forward pass (lane b): bias acceleration and body forces
  float r_cfrc[6];
  {
    const float g0 = -m.gravity_x, g1 = -m.gravity_y, g2 = -m.gravity_z;
    float a[6] = {0.f, 0.f, 0.f, g0, g1, g2};
    for (int j = 0; j < nv; j++) {
      const float q = ((r_dm >> j) & 1ull) ? rl(r_qv, j) : 0.f;
#pragma unroll
      for (int c = 0; c < 6; c++) a[c] += rl(r_cdd[c], j) * q;
    }
    float f1[6], f2[6], f3[6];
    inert_vec(f1, r_cin, a);
    inert_vec(f2, r_cin, r_cvel);
    cross_force(f3, r_cvel, f2);
#pragma unroll
    for (int c = 0; c < 6; c++) r_cfrc[c] = (tid == 0) ? 0.f : f1[c] + f3[c];
  }
  PROF(23);
  // subtree sums of cfrc (lane b), ascending k
  float r_bf[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, r_bias = 0.f;
#pragma nounroll
  for (int k = 1; k < nb; k++) {
    const float in = (tid > 0 && ((rl64(r_tmk, k) >> tid) & 1ull)) ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < 6; c++) r_bf[c] = fmaf(rl(r_cfrc[c], k), in, r_bf[c]);
  }
  if (bl) {
#pragma unroll
    for (int c = 0; c < 6; c++) cfrc[6 * tid + c] = r_cfrc[c];
  }
  {
    const int bi = tid < nv ? IMG_I(dof_bodyid)[tid] : 0;
    float f[6];
#pragma unroll
    for (int c = 0; c < 6; c++) f[c] = shfl(r_bf[c], bi);
    if (tid < nv) {
      const float* cd = r_cdof;
      r_bias = cd[0] * f[0] + cd[1] * f[1] + cd[2] * f[2] + cd[3] * f[3] + cd[4] * f[4] + cd[5] * f[5];
      qfrc_bias[tid] = r_bias;
    }
  }
  wsync();

  PROF(24);
  // ---------------------------------------------------------------- passive, actuation, smooth force
  // lane i = dof i (nv < 64); passive force and bias stay in registers, the
  // applied force is loaded before any store
  const float r_qapp = tid < nv ? DP(qfrc_applied)[W * nv + tid] : 0.f;
  float r_pas = 0.f;
  if (tid < nv) {
    const int i = tid;
    float pas = -dof_damping[i] * qvel[i];
    const int jnt = IMG_I(dof_jntid)[i];
    const int t = IMG_I(jnt_type)[jnt];
    if ((t == 2 || t == 3) && jnt_stiffness[jnt] != 0.f) {
      const int qa = IMG_I(jnt_qposadr)[jnt];
      pas -= jnt_stiffness[jnt] * (qpos[qa] - IMG_F(qpos_spring)[qa]);
    } else if (t == 1 && jnt_stiffness[jnt] != 0.f) {  // ball: the rotation vector from the spring pose
      const int qa = IMG_I(jnt_qposadr)[jnt], k = i - IMG_I(jnt_dofadr)[jnt];
      float dif[3];
      sub_quat(dif, qpos + qa, IMG_F(qpos_spring) + qa);
      pas -= jnt_stiffness[jnt] * (k == 0 ? dif[0] : (k == 1 ? dif[1] : dif[2]));
    }
    qfrc_passive[i] = pas;
    qfrc_act[i] = 0.f;
    r_pas = pas;
  }
  wsync();
  for (int i = tid; i < nu; i += NT) {
    const int j = IMG_I(actuator_trnid)[i];
    const float gear = IMG_F(actuator_gear)[i];
    const float len = gear * qpos[IMG_I(jnt_qposadr)[j]];
    const float vel = gear * qvel[IMG_I(jnt_dofadr)[j]];
    float c = DP(ctrl)[W * nu + i];
    if (IMG_I(actuator_ctrllimited)[i]) c = clampf(c, IMG_F(actuator_ctrlrange)[2 * i], IMG_F(actuator_ctrlrange)[2 * i + 1]);
    const float* gp = IMG_F(actuator_gainprm) + 10 * i;
    const float* bp = IMG_F(actuator_biasprm) + 10 * i;
    float f = gp[0] * c + bp[0] + bp[1] * len + bp[2] * vel;
    if (IMG_I(actuator_forcelimited)[i]) f = clampf(f, IMG_F(actuator_forcerange)[2 * i], IMG_F(actuator_forcerange)[2 * i + 1]);
    act_force[i] = f;
    DP(actuator_force)[W * nu + i] = f;
    DP(actuator_length)[W * nu + i] = len;
    DP(actuator_velocity)[W * nu + i] = vel;
    // one actuator per dof in mjlab models; atomic keeps it correct otherwise
    atomicAdd(&qfrc_act[IMG_I(jnt_dofadr)[j]], gear * f);
  }
  wsync();
  {
    const float* xfrc = DP(xfrc_applied) + W * nb * 6;
    // bodies with a nonzero applied wrench, found with one load round (lane =
    // body) instead of a dependent global-load chain per dof
    bool nzf = false;
    if (tid > 0 && tid < nb) {
      const float* f = xfrc + 6 * tid;
      nzf = f[0] != 0.f || f[1] != 0.f || f[2] != 0.f || f[3] != 0.f || f[4] != 0.f || f[5] != 0.f;
    }
    const unsigned long long nzb = __ballot(nzf);
    for (int i = tid; i < nv; i += NT) {
      float s = r_pas - r_bias + r_qapp + qfrc_act[i];
      // J^T xfrc_applied at each body com
      const float* cd = cdof + 6 * i;
      for (unsigned long long bm = nzb; bm; bm &= bm - 1) {
        const int b = __builtin_ctzll(bm);
        if (!(((unsigned long long)IMG_L(body_dofmask)[b] >> i) & 1ull)) continue;
        const float* f = xfrc + 6 * b;
        const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
        float off[3] = {xipos[3 * b] - c[0], xipos[3 * b + 1] - c[1], xipos[3 * b + 2] - c[2]}, t[3];
        cross3(t, cd, off);
        s += (cd[3] + t[0]) * f[0] + (cd[4] + t[1]) * f[1] + (cd[5] + t[2]) * f[2] + cd[0] * f[3] + cd[1] * f[4] + cd[2] * f[5];
      }
      qfrc_smooth[i] = s;
      qacc_smooth[i] = s;
    }
  }
  PROF(25);
  ldl_solve_reg<NVP, PKL>(MODE == 2 ? G + Lo.h_L : Lm, nv, ldm, qacc_smooth);
  PROF(3);

  // ---------------------------------------------------------------- Newton solver
  const float scale = 1.f / (m.meaninertia * (float)(nv > 1 ? nv : 1));
  int niter = 0, nfactor_total = 0;
  // solver_lstrace: the parallel line search's step-size index (6 bits) of
  // iterations 5w..5w+4 in word w (15 iterations), bit 30 of word 0: the solve
  // started from qacc_smooth, bit 30 of word 1: the last iteration passed the
  // convergence test (the parity tests replay the choices and check both
  // decisions against the oracle's own)
  unsigned lstr0 = 0u, lstr1 = 0u, lstr2 = 0u;
  if (nefc == 0) {
    for (int i = tid; i < nv; i += NT) {
      qacc[i] = qacc_smooth[i];
      qfrc_con[i] = 0.f;
    }
    wsync();
  } else {
    // forces, qfrc_constraint and cost at the point whose jaref / Ma are set
    // elliptic cones: the contact's rows, gathered by the lane of its first
    // row (rows of other contacts' lanes are skipped there); at step a along jv
    auto cone_first = [&](int r, int& dim) -> bool {
      const int ci = efc_id[r];
      dim = con_dim[ci];
      return con_efcadr[ci] == r;
    };
    auto cone_load = [&](int r0, int dim, const float* x, float a, ConeRows& c, float* jvv) {
#pragma unroll
      for (int j = 0; j < 6; j++) {
        const int rj = j < dim ? r0 + j : r0;
        c.jar[j] = x[rj] + a * jv[rj];
        c.D[j] = efc_D[rj];
        c.s[j] = efc_fl[rj];
        if (jvv) jvv[j] = jv[rj];
      }
    };
    auto update_constraint = [&]() -> float {
      float c = 0.f;
#if MJH_JTF_PF
      // J^T f's first round of J loads issued before the row pass (they do not
      // depend on it): one global round trip off the update's chain
      float jpf[MJH_JTF_B];
      const bool pf = nefc >= MJH_JTF_B;
      if (pf) {
        const int ic = tid < nv ? tid : 0;
#pragma unroll
        for (int q = 0; q < MJH_JTF_B; q++) jpf[q] = J[q * ldj + ic];
      }
#endif
      for (int r = tid; r < nefc; r += NT) {
        float f, cr;
        if (ELL && efc_type[r] == MJH_CNSTR_CONTACT_ELLIPTIC) {
          int dim;
          if (!cone_first(r, dim)) continue;
          ConeRows cr6;
          cone_load(r, dim, jaref, 0.f, cr6, nullptr);
          float fc[6];
          int zone;
          c += cone_eval(dim, cr6, fc, &zone);
          // Hessian weights: bottom zone per row; the cone's block is added by
          // newton_direction as virtual rows (marked by -1 on the first row)
#pragma unroll
          for (int j = 0; j < 6; j++)
            if (j < dim) {
              efc_force[r + j] = fc[j];
              efc_h[r + j] = zone == kConeBottom ? cr6.D[j] : (zone == kConeMid && j == 0 ? -1.f : 0.f);
            }
          continue;
        }
        efc_h[r] = row_state(efc_type[r], efc_D[r], efc_R[r], efc_fl[r], jaref[r], &f, &cr);
        efc_force[r] = f;
        c += cr;
      }
      for (int i = tid; i < nv; i += NT) c += 0.5f * (Ma[i] - qfrc_smooth[i]) * (qacc[i] - qacc_smooth[i]);
      wsync();
      for (int i = tid; i < nv; i += NT) {
        // J^T f: entries outside a row's dof mask are exact zeros, so no test.
        // MJH_JTF_B rows of J loads in flight per round; accumulator k takes rows r = k
        // mod 4 in increasing order (as a plain 4-way unrolled loop)
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int r = 0;
#if MJH_JTF_PF
        if (pf) {
#pragma unroll
          for (int q = 0; q < MJH_JTF_B; q += 4) {
            s0 += jpf[q] * efc_force[q];
            s1 += jpf[q + 1] * efc_force[q + 1];
            s2 += jpf[q + 2] * efc_force[q + 2];
            s3 += jpf[q + 3] * efc_force[q + 3];
          }
          r = MJH_JTF_B;
        }
#endif
        for (; r + MJH_JTF_B <= nefc; r += MJH_JTF_B) {
          float jj[MJH_JTF_B];
#pragma unroll
          for (int q = 0; q < MJH_JTF_B; q++) jj[q] = J[(r + q) * ldj + i];
#pragma unroll
          for (int q = 0; q < MJH_JTF_B; q += 4) {
            s0 += jj[q] * efc_force[r + q];
            s1 += jj[q + 1] * efc_force[r + q + 1];
            s2 += jj[q + 2] * efc_force[r + q + 2];
            s3 += jj[q + 3] * efc_force[r + q + 3];
          }
        }
        for (; r + 4 <= nefc; r += 4) {
          s0 += J[r * ldj + i] * efc_force[r];
          s1 += J[(r + 1) * ldj + i] * efc_force[r + 1];
          s2 += J[(r + 2) * ldj + i] * efc_force[r + 2];
          s3 += J[(r + 3) * ldj + i] * efc_force[r + 3];
        }
        for (; r < nefc; r++) s0 += J[r * ldj + i] * efc_force[r];
        qfrc_con[i] = (s0 + s1) + (s2 + s3);
      }
      return bsum<NT>(c, red);
    };
    // active set of the factor in Lm as wave-uniform row masks (no memory: a
    // global copy of the row list put a store ahead of the next J loads)
    constexpr int kMaskWords = 5;  // rows beyond 320: always rebuild
    unsigned long long act_prev[kMaskWords] = {0ull, 0ull, 0ull, 0ull, 0ull};
    bool have_prev = false, cone_prev = false;
    int nfactor = 0;
    // gradient at the current point (the convergence test reads only this)
    auto gradient = [&]() {
      for (int i = tid; i < nv; i += NT) grad[i] = Ma[i] - qfrc_smooth[i] - qfrc_con[i];
    };
    // Newton direction from grad: Hessian (kept while the active set is
    // unchanged), factor, solve
    auto newton_direction = [&]() {
      // compact the rows in the quadratic zone: H = M + sum h_r J_r J_r^T
      int nact = 0;
      unsigned long long act[kMaskWords] = {0ull, 0ull, 0ull, 0ull, 0ull};
      for (int base = 0; base < nefc; base += NT) {
        const int r = base + tid;
        const float h = r < nefc ? efc_h[r] : 0.f;
        const int a = h > 0.f ? 1 : 0;
        const unsigned long long bal = __ballot(a);
#pragma unroll
        for (int q = 0; q < kMaskWords; q++) act[q] = q == base / NT ? bal : act[q];
        int total;
        const int off = bscan<NT>(a, &total, redi);
        if (a) {
          if (MJH_BOK(nact + off, acap + 4)) {
            arow[nact + off] = r;
            ash[nact + off] = sqrtf(h);
          }
        }
        nact += total;
      }
      wsync();
      // elliptic contacts in the cone zone (efc_h -1 on the first row): their
      // Hessian block Hc = a a^T + sum_q b_q b_q^T (a = sqrt(Dm) S grad(N - mu T),
      // b_q = sqrt(Dm mu (mu T - N) / T) S e_q, e_q an orthonormal basis of the
      // tangent plane's complement of U / T from a Householder reflection) as
      // virtual rows sum_j coef_j J_{r0+j}, stored after row rcap
      int ncone = 0;
      if (ELL) {
        for (int base = 0; base < nefc; base += NT) {
          const int rr = base + tid;
          unsigned long long bal = __ballot(rr < nefc && efc_h[rr] < 0.f);
          while (bal) {
            const int r0 = base + __builtin_ctzll(bal);
            bal &= bal - 1ull;
            int dim;
            (void)cone_first(r0, dim);
            ConeRows c;
            cone_load(r0, dim, jaref, 0.f, c, nullptr);
            const float mu = c.s[0];
            float U[6], TT = 0.f;
#pragma unroll
            for (int j = 1; j < 6; j++) {
              U[j] = j < dim ? c.jar[j] * c.s[j] : 0.f;
              TT += U[j] * U[j];
            }
            const float N = c.jar[0] * mu, T = sqrtf(TT);
            const float Dm = c.D[0] / fmaxf(mu * mu * (1.f + mu * mu), MJH_MINVAL);
            const float sa = sqrtf(Dm), sb = sqrtf(fmaxf(Dm * mu * (mu * T - N) / T, 0.f));
            // Householder v = u + sign(u1) e1 over the tangent dims 1..dim-1
            float v[6], vv = 0.f;
#pragma unroll
            for (int j = 1; j < 6; j++) v[j] = j < dim ? U[j] / T : 0.f;
            v[1] += v[1] >= 0.f ? 1.f : -1.f;
#pragma unroll
            for (int j = 1; j < 6; j++) vv += v[j] * v[j];
#pragma unroll
            for (int q = 0; q < 5; q++) {
              if (q >= dim - 1) break;
              float cf[6];
              cf[0] = q == 0 ? sa * mu : 0.f;
#pragma unroll
              for (int j = 1; j < 6; j++) {
                // q = 0: -sqrt(Dm) mu u_j s_j; q >= 1: sb e_q[j] s_j, e_q column q+1 of I - 2 v v^T / |v|^2
                const float eq = (j == q + 1 ? 1.f : 0.f) - 2.f * v[j] * v[q + 1 < 6 ? q + 1 : 5] / vv;
                cf[j] = j >= dim ? 0.f : (q == 0 ? -sa * mu * (U[j] / T) * c.s[j] : sb * eq * c.s[j]);
              }
              const int vr = Lo.rcap + ncone;
              if (tid < ldj) {
                float val = 0.f;
#pragma unroll
                for (int j = 0; j < 6; j++)
                  if (j < dim) val += cf[j] * J[(r0 + j) * ldj + tid];
                if (MJH_BOK(vr, m.cone == 1 ? 2 * Lo.rcap : Lo.rcap)) J[vr * ldj + tid] = val;
              }
              if (tid == 0) {
                if (MJH_BOK(nact, acap + 4)) {
                  arow[nact] = vr;
                  ash[nact] = 1.f;
                }
              }
              nact++;
              ncone++;
            }
          }
        }
        wsync();
      }
      // same active set as the factor in Lm -> H is identical, keep the factor
      // (never with cone-zone contacts: their blocks move with jar)
      bool same = have_prev && nefc <= kMaskWords * NT && ncone == 0 && !cone_prev;
#pragma unroll
      for (int q = 0; q < kMaskWords; q++) same = same && act[q] == act_prev[q];
      float diff = same ? 0.f : 1.f;
#ifdef MJH_DEBUG_ALWAYS_REBUILD
      diff = 1.f;
#endif
      if (diff != 0.f) {
        unsigned long long th = PROF_NOW();
#ifdef MJH_DEBUG_PLAIN_HESSIAN
        wsync();
        for (int i = tid; i < nv; i += NT)
          for (int j = 0; j <= i; j++) {
            float hs = Mm[i * ldm + j];
            for (int k = 0; k < nact; k++) hs += ash[k] * ash[k] * J[arow[k] * ldj + i] * J[arow[k] * ldj + j];
            Lm[lofs<PKL>(i, ldm) + j] = hs;
          }
#else
        hessian_mfma<NT, NVP, PKL>(Mm, ldm, J, ldj, arow, ash, nact, nv, Lm);
#endif
        PROF_ACC(15, th);
        unsigned long long tf = PROF_NOW();
#if MJH_FUSED_FWD
        for (int i = tid; i < nv; i += NT) search[i] = grad[i];
        ldl_factor_solve_reg<NVP, PKL>(Lm, nv, ldm, search);
#else
        ldl_factor_reg<NVP, PKL>(Lm, nv, ldm);
#endif
        PROF_ACC(16, tf);
#pragma unroll
        for (int q = 0; q < kMaskWords; q++) act_prev[q] = act[q];
        have_prev = true;
        cone_prev = ncone > 0;
        nfactor++;
        nfactor_total++;
      }
      unsigned long long ts = PROF_NOW();
      if (!MJH_FUSED_FWD || diff == 0.f) {  // a kept factor: the plain solve
        for (int i = tid; i < nv; i += NT) search[i] = grad[i];
        ldl_solve_reg<NVP, PKL>(Lm, nv, ldm, search);
      }
      PROF_ACC(17, ts);
      for (int i = tid; i < nv; i += NT) search[i] = -search[i];
      wsync();
    };

    // CG (opt.solver == mjSOL_CG): MuJoCo's primal solver with the search
    // direction from M instead of the Hessian (engine_solver.c mj_solPrimal,
    // MuJoCo Warp solver.py): Mgrad = M^-1 grad through M's factor (still in
    // Lm: CG never builds a Hessian), the first search -Mgrad, later ones
    // Polak-Ribiere: search = -Mgrad + max(0, beta) search with beta =
    // grad.(Mgrad - Mgrad_old) / max(mjMINVAL, grad_old.Mgrad_old)
    const bool use_cg = m.solver == kSolverCG;
    float* const Mgrad = tmp;
    float* const cg_g = SP(cg_g);
    float* const cg_mg = SP(cg_mg);
    auto cg_direction = [&](bool first) {
      for (int i = tid; i < nv; i += NT) Mgrad[i] = grad[i];
      ldl_solve_reg<NVP, PKL>(MODE == 2 ? G + Lo.h_L : Lm, nv, ldm, Mgrad);  // M's factor
      float num = 0.f, den = 0.f;
      if (!first) {
        for (int i = tid; i < nv; i += NT) {
          num += grad[i] * (Mgrad[i] - cg_mg[i]);
          den += cg_g[i] * cg_mg[i];
        }
        bsum2<NT>(num, den, red);
      }
      const float beta = first ? 0.f : fmaxf(0.f, num / fmaxf(MJH_MINVAL, den));
      for (int i = tid; i < nv; i += NT) {
        const float mg = Mgrad[i];
        search[i] = first ? -mg : -mg + beta * search[i];
        cg_g[i] = grad[i];
        cg_mg[i] = mg;
      }
      wsync();
    };
    auto direction = [&](bool first) {
      if (use_cg)
        cg_direction(first);
      else
        newton_direction();
    };

    // PGS (opt.solver == mjSOL_PGS; generic instances only): MuJoCo's projected
    // Gauss-Seidel on the dual (engine_solver.c mj_solPGS with the dual warm
    // start of engine_forward.c; MuJoCo Warp has no PGS). The oracle's
    // solve_pgs is the restatement this follows: minimise 0.5 f'AR f + f'b,
    // AR = J M^-1 J' + diag(R), b = J qacc_smooth - aref (kept in jv), one row
    // at a time with projection and the undo of a cost-increasing update; the
    // sweep's improvement ends the solve. AR and the rows M^-1 J_r' live in
    // global scratch (Lo.pgs_ar, Lo.pgs_mj), M's factor is still in Lm.
    bool pgs = false;
    if constexpr (SPEC < 0) pgs = m.solver == kSolverPGS;
    if (pgs) {
      float* const AR = G + Lo.pgs_ar;
      float* const MJ = G + Lo.pgs_mj;
      const int lda = Lo.rcap;
      const float* const Lf = MODE == 2 ? G + Lo.h_L : Lm;
      for (int r = 0; r < nefc; r++) {
        for (int i = tid; i < nv; i += NT) tmp[i] = J[r * ldj + i];
        ldl_solve_reg<NVP, PKL>(Lf, nv, ldm, tmp);
        for (int i = tid; i < ldj; i += NT) MJ[r * ldj + i] = i < nv ? tmp[i] : 0.f;
      }
      wsync();
      for (int i = 0; i < nefc; i++)
        for (int j = tid; j < nefc; j += NT) AR[i * lda + j] = rowdot_u<NVP>(J + i * ldj, MJ + j * ldj, nv) + (j == i ? efc_R[i] : 0.f);
      for (int r = tid; r < nefc; r += NT) jv[r] = rowdot_u<NVP>(J + r * ldj, qacc_smooth, nv) - efc_aref[r];
      // warm start: the forces of qacc_warmstart's constraint state, zero when
      // their dual cost is positive
      for (int i = tid; i < nv; i += NT) qacc[i] = DP(qacc_warmstart)[W * nv + i];
      wsync();
      for (int r = tid; r < nefc; r += NT) {
        float f, cr;
        row_state(efc_type[r], efc_D[r], efc_R[r], efc_fl[r], rowdot_u<NVP>(J + r * ldj, qacc, nv) - efc_aref[r], &f, &cr);
        efc_force[r] = f;
      }
      wsync();
      float wc = 0.f;
      for (int r = tid; r < nefc; r += NT) {
        float af = 0.f;
        for (int j = 0; j < nefc; j++) af += AR[r * lda + j] * efc_force[j];
        wc += efc_force[r] * (jv[r] + 0.5f * af);
      }
      wc = bsum<NT>(wc, red);
      if (wc > 0.f) {
        lstr0 |= 1u << 30;
        for (int r = tid; r < nefc; r += NT) efc_force[r] = 0.f;
      }
      wsync();
      for (int it = 0; it < m.iterations; it++) {
        float improvement = 0.f;
        for (int i = 0; i < nefc; i++) {
          float sres = 0.f;
          for (int j = tid; j < nefc; j += NT) sres += AR[i * lda + j] * efc_force[j];
          const float res = jv[i] + bsum<NT>(sres, red);
          const float aii = AR[i * lda + i], old = efc_force[i];
          float fi = old - res / fmaxf(aii, MJH_MINVAL);
          if (efc_type[i] == MJH_CNSTR_FRICTION_DOF) {
            const float fl = efc_fl[i];
            fi = fi < -fl ? -fl : (fi > fl ? fl : fi);
          } else if (fi < 0.f) {
            fi = 0.f;
          }
          const float dl = fi - old;
          float change = 0.5f * dl * dl * aii + dl * res;
          if (change > 1e-10f) {
            fi = old;
            change = 0.f;
          }
          improvement -= change;
          wsync();
          if (tid == 0) efc_force[i] = fi;
          wsync();
        }
        niter++;
        if (improvement * scale < m.tolerance) {
          lstr1 |= 1u << 30;
          break;
        }
      }
      for (int i = tid; i < nv; i += NT) {
        float sf = 0.f;
        for (int r = 0; r < nefc; r++) sf += J[r * ldj + i] * efc_force[r];
        qfrc_con[i] = sf;
        tmp[i] = sf;
      }
      ldl_solve_reg<NVP, PKL>(Lf, nv, ldm, tmp);
      for (int i = tid; i < nv; i += NT) qacc[i] = qacc_smooth[i] + tmp[i];
      wsync();
    } else {
    // warm start: the cheaper of qacc_warmstart and qacc_smooth, both
    // evaluated in one pass over M's and J's rows (each row loaded once; the
    // qacc_smooth values wait in Mv / jv in case they win)
    for (int i = tid; i < nv; i += NT) qacc[i] = DP(qacc_warmstart)[W * nv + i];
    wsync();
    for (int i = tid; i < nv; i += NT) rowdot2_u<NVP>(Mm + i * ldm, qacc, qacc_smooth, nv, Ma[i], Mv[i]);
    for (int r = tid; r < nefc; r += NT) {
      float a, b;
      rowdot2_u<NVP>(J + r * ldj, qacc, qacc_smooth, nv, a, b);
      jaref[r] = a - efc_aref[r];
      jv[r] = b - efc_aref[r];
    }
    wsync();
    float cost = update_constraint();
    float cs = 0.f;
    for (int r = tid; r < nefc; r += NT) {
      float f, cr;
      if (ELL && efc_type[r] == MJH_CNSTR_CONTACT_ELLIPTIC) {
        int dim;
        if (!cone_first(r, dim)) continue;
        ConeRows c;
        cone_load(r, dim, jv, 0.f, c, nullptr);
        float fc[6];
        int zone;
        cs += cone_eval(dim, c, fc, &zone);
        continue;
      }
      row_state(efc_type[r], efc_D[r], efc_R[r], efc_fl[r], jv[r], &f, &cr);
      cs += cr;
    }
    const float cost_smooth = bsum<NT>(cs, red);
    if (cost > cost_smooth) lstr0 |= 1u << 30;
    if (cost > cost_smooth) {
      for (int i = tid; i < nv; i += NT) {
        qacc[i] = qacc_smooth[i];
        Ma[i] = Mv[i];
      }
      for (int r = tid; r < nefc; r += NT) jaref[r] = jv[r];
      wsync();
      cost = update_constraint();
    }
    wsync();
    gradient();
    direction(true);

    for (int it = 0; it < m.iterations; it++) {
      unsigned long long t_ls = PROF_NOW();
      // a world still iterating raises its wave's issue priority (the launch ends
      // with its slowest world; the SIMD's other waves fill in). Measured
      // (profiles/r05a_prio_kb.log): Go1 8192 0.457 -> 0.449 ms, G1 4096 0.501 ->
      // 0.511 ms, so on for models up to 20 dofs only (MJH_PRIO: 1 all, 0 none)
      if constexpr (MJH_PRIO == 1 || (MJH_PRIO < 0 && NVP <= 20)) {
        if (it == 2) __builtin_amdgcn_s_setprio(1);
        if (it == 4) __builtin_amdgcn_s_setprio(2);
        if (it == 6) __builtin_amdgcn_s_setprio(3);
      }
      // ---- exact line search along `search`
      symv_u<NT, NVP>(Mm, nv, ldm, search, Mv);
      for (int r = tid; r < nefc; r += NT) {
        jv[r] = rowdot_u<NVP>(J + r * ldj, search, nv);
      }
      wsync();
      float g1 = 0.f, g2 = 0.f;
      for (int i = tid; i < nv; i += NT) {
        g1 += search[i] * (Ma[i] - qfrc_smooth[i]);
        g2 += search[i] * Mv[i];
      }
      bsum2<NT>(g1, g2, red);
      auto derivs = [&](float alpha, float& d1, float& d2) {
        float a = 0.f, b = 0.f;
        for (int r = tid; r < nefc; r += NT) {
          float f, cr;
          if (ELL && efc_type[r] == MJH_CNSTR_CONTACT_ELLIPTIC) {
            int dim;
            if (!cone_first(r, dim)) continue;
            ConeRows c;
            float jvv[6], fc[6], q2;
            int zone;
            cone_load(r, dim, jaref, alpha, c, jvv);
            cone_eval(dim, c, fc, &zone, jvv, &q2);
#pragma unroll
            for (int j = 0; j < 6; j++) a -= j < dim ? fc[j] * jvv[j] : 0.f;
            b += q2;
            continue;
          }
          const float h = row_state(efc_type[r], efc_D[r], efc_R[r], efc_fl[r], jaref[r] + alpha * jv[r], &f, &cr);
          a -= f * jv[r];
          b += h * jv[r] * jv[r];
        }
        bsum2<NT>(a, b, red);
        d1 = g1 + alpha * g2 + a;
        d2 = g2 + b;
      };
      float alpha = 0.f;
      if (m.ls_parallel) {
        // MuJoCo Warp's parallel line search (solver.py, linesearch_parallel):
        // the cost at nlsp = ls_iterations step sizes log-spaced over
        // [ls_parallel_min_step, 1]; the cheapest wins (the smallest on ties).
        const int nlsp = m.ls_iterations;
        const float lmin = logf(m.ls_parallel_min_step);
        const float lstep = (0.f - lmin) / fmaxf(1.f, (float)(nlsp - 1));
        float best = INFINITY;
        int bi = 0;
        if (nefc <= 2 * NT && !ELL) {
          // a lane's (at most two) rows in registers, loaded once; four step
          // sizes per block, their four wave reductions independent (the
          // reduction latency overlaps instead of serialising per step size)
          int ty[2];
          float rD[2], rR[2], rf[2], rj[2], rv[2];
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const int r = tid + q * NT;
            const bool in = r < nefc;
            ty[q] = in ? efc_type[r] : -1;
            rD[q] = in ? efc_D[r] : 0.f;
            rR[q] = in ? efc_R[r] : 0.f;
            rf[q] = in ? efc_fl[r] : 0.f;
            rj[q] = in ? jaref[r] : 0.f;
            rv[q] = in ? jv[r] : 0.f;
          }
          // row cost at step a (row_state's cost, branch-free selects)
          auto rcost = [&](int q, float a) -> float {
            const float x = rj[q] + a * rv[q];
            const float quad = 0.5f * rD[q] * x * x;
            if (ty[q] == MJH_CNSTR_FRICTION_DOF) {
              const float lim = rR[q] * rf[q], k = 0.5f * rR[q] * rf[q] * rf[q];
              return x >= lim ? rf[q] * x - k : (x <= -lim ? -rf[q] * x - k : quad);
            }
            return (ty[q] >= 0 && x < 0.f) ? quad : 0.f;
          };
          // The cost is convex in the step size (a convex quadratic plus
          // convex piecewise-quadratic rows), so its first minimiser on the
          // increasing grid is found scanning down from the largest step and
          // stopping at the first increase — the same index as evaluating
          // all nlsp (ties go to the smaller step), usually after one pair,
          // since the full Newton step (1) mostly wins.
          bi = nlsp - 1;
          for (int k = nlsp - 1; k >= 0; k -= 2) {
            const float a0 = expf(lmin + (float)k * lstep), a1 = expf(lmin + (float)(k - 1) * lstep);
            float c0 = rcost(0, a0) + rcost(1, a0), c1 = rcost(0, a1) + rcost(1, a1);
            bsum2<NT>(c0, c1, red);
            c0 += a0 * (g1 + 0.5f * a0 * g2);
            c1 += a1 * (g1 + 0.5f * a1 * g2);
            if (!(c0 <= best)) break;
            best = c0;
            bi = k;
            if (k - 1 < 0 || !(c1 <= best)) break;
            best = c1;
            bi = k - 1;
          }
        } else
        for (int k = 0; k < nlsp; k += 2) {
          const float aa = expf(lmin + (float)k * lstep), ab = expf(lmin + (float)(k + 1) * lstep);
          float ca = 0.f, cb = 0.f;
          for (int r = tid; r < nefc; r += NT) {
            float f, cr;
            if (ELL && efc_type[r] == MJH_CNSTR_CONTACT_ELLIPTIC) {
              int dim;
              if (!cone_first(r, dim)) continue;
              ConeRows c;
              float fc[6];
              int zone;
              cone_load(r, dim, jaref, aa, c, nullptr);
              ca += cone_eval(dim, c, fc, &zone);
              cone_load(r, dim, jaref, ab, c, nullptr);
              cb += cone_eval(dim, c, fc, &zone);
              continue;
            }
            const float ja = jaref[r], j1 = jv[r];
            row_state(efc_type[r], efc_D[r], efc_R[r], efc_fl[r], ja + aa * j1, &f, &cr);
            ca += cr;
            row_state(efc_type[r], efc_D[r], efc_R[r], efc_fl[r], ja + ab * j1, &f, &cr);
            cb += cr;
          }
          bsum2<NT>(ca, cb, red);
          ca += aa * (g1 + 0.5f * aa * g2);
          cb += ab * (g1 + 0.5f * ab * g2);
#ifdef MJH_PROFILE
          // diagnostics: candidate costs at iteration MJH_LSDBG_IT into free profile slots
          if (tid == 0 && g_lsdbg && it == MJH_LSDBG_IT && k + 1 < 32) {
            g_lsdbg[(long long)w * 32 + k] = ca;
            if (k + 1 < nlsp) g_lsdbg[(long long)w * 32 + k + 1] = cb;
          }
#endif
          if (ca < best) { best = ca; bi = k; }
          if (k + 1 < nlsp && cb < best) { best = cb; bi = k + 1; }
        }
        alpha = expf(lmin + (float)bi * lstep);
        if (it < 5) lstr0 |= (unsigned)(bi & 63) << (6 * it);
        else if (it < 10) lstr1 |= (unsigned)(bi & 63) << (6 * (it - 5));
        else if (it < 15) lstr2 |= (unsigned)(bi & 63) << (6 * (it - 10));
      } else {
      float d10, d20;
      derivs(0.f, d10, d20);
      if (d10 < 0.f) {
        const float gtol = m.ls_tolerance * fabsf(d10);
        float lo = 0.f, hi = -1.f;
        alpha = -d10 / d20;
        for (int li = 0; li < m.ls_iterations; li++) {
          float d1, d2;
          derivs(alpha, d1, d2);
          if (fabsf(d1) <= gtol) break;
          if (d1 < 0.f) lo = alpha; else hi = alpha;
          float an = alpha - d1 / d2;
          if (an <= lo || (hi >= 0.f && an >= hi)) an = hi >= 0.f ? 0.5f * (lo + hi) : 2.f * alpha;
          alpha = an;
        }
      }
      }
      PROF_ACC(12, t_ls);
      if (alpha == 0.f) break;
      unsigned long long t_up = PROF_NOW();
      for (int i = tid; i < nv; i += NT) {
        qacc[i] += alpha * search[i];
        Ma[i] += alpha * Mv[i];
      }
      for (int r = tid; r < nefc; r += NT) jaref[r] += alpha * jv[r];
      wsync();
      const float old = cost;
      cost = update_constraint();
      wsync();
      PROF_ACC(13, t_up);
      gradient();
      niter++;
      float gn = 0.f;
      for (int i = tid; i < nv; i += NT) gn += grad[i] * grad[i];
      gn = bsum<NT>(gn, red);
      const float improvement = scale * (old - cost), gnorm = scale * sqrtf(gn);
      if (improvement < m.tolerance || gnorm < m.tolerance) {
        lstr1 |= 1u << 30;  // stopped by the convergence test (the parity tests check this decision)
        break;
      }
      // the direction is read only by a further iteration: none after the last
      // (MuJoCo / MuJoCo Warp compute it before the test; nothing reads it after)
      if (it + 1 >= m.iterations) break;
      unsigned long long t_nd = PROF_NOW();
      direction(false);
      PROF_ACC(14, t_nd);
    }
    }  // Newton / CG
  }
  wsync();

  // ---------------------------------------------------------------- post-constraint acceleration (cacc)
  PROF(6);
#ifdef MJH_PROFILE
  if (tid == 0 && g_prof) g_prof[(long long)w * 32 + 29] = (unsigned long long)nfactor_total;
#endif
  {
    // lane b: sum over the dofs j of b's chain (ascending), lane j's rows via readlane
    const float g0 = -m.gravity_x, g1 = -m.gravity_y, g2 = -m.gravity_z;
    float cd[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, cdd[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float qv_l = 0.f, qa_l = 0.f;
    if (tid < nv) {
#pragma unroll
      for (int c = 0; c < 6; c++) { cd[c] = cdof[6 * tid + c]; cdd[c] = cdof_dot[6 * tid + c]; }
      qv_l = qvel[tid]; qa_l = qacc[tid];
    }
    const unsigned long long dm = bl ? dmk[tid] : 0ull;
    float a[6] = {0.f, 0.f, 0.f, g0, g1, g2};
#if MJH_CACC_W
    // lane j forms its own term cdof_dot_j qvel_j + cdof_j qacc_j; the chain sum
    // then reads 6 values per dof instead of 14
    float wv[6];
#pragma unroll
    for (int c = 0; c < 6; c++) wv[c] = cdd[c] * qv_l + cd[c] * qa_l;
    for (int j = 0; j < nv; j++) {
      const bool in = (dm >> j) & 1ull;
#pragma unroll
      for (int c = 0; c < 6; c++) {
        const float t = rl(wv[c], j);
        a[c] += in ? t : 0.f;
      }
    }
#else
    for (int j = 0; j < nv; j++) {
      const bool in = (dm >> j) & 1ull;
      const float qv = in ? rl(qv_l, j) : 0.f, qa = in ? rl(qa_l, j) : 0.f;
#pragma unroll
      for (int c = 0; c < 6; c++) {
        const float x = rl(cdd[c], j), y = rl(cd[c], j);
        a[c] += x * qv + y * qa;
      }
    }
#endif
    if (bl) {
#pragma unroll
      for (int c = 0; c < 6; c++) cacc[6 * tid + c] = a[c];
    }
  }
  wsync();
  PROF(26);

  // ---------------------------------------------------------------- sensors
  {
    float* sd = DP(sensordata) + W * Z.nsensordata;
    // contact tid's force (contact frame, mj_contactForce for pyramidal cones),
    // frame, position, distance and geoms in registers, loaded once for all
    // contact sensors when ncon <= 64 (then a sensor's kept matches fetch them
    // by ds_bpermute instead of a dependent chain of scratch loads)
    const bool creg = ncon <= 64;
    bool cloaded = false;
    float cF[6], cfr[9], cps[3], cds = 0.f;
    int cg1 = 0, cg2 = 0, cb1 = 0, cb2 = 0;  // contact tid's geoms and their bodies
    unsigned long long ct1 = 0ull, ct2 = 0ull;  // the bodies' subtree masks (body_treemask)
    // the sensors' metadata, lane s = sensor s (< 64), loaded in one round instead
    // of a dependent chain of loads per sensor; read back by readlane (uniform s)
    // (MJH_SENS_PRELOAD: 0 per-sensor loads, 1 one register per field, 2 packed
    // into four registers; measured in profiles/r06*_ab)
#if MJH_SENS_PRELOAD == 1
    int q_type = -1, q_id = 0, q_adr = 0, q_bits = 0, q_red = 0, q_nslot = 0, q_ot = 0, q_rt = 0, q_rid = 0, q_dim = 0;
    if (tid < Z.nsensor) {
      q_type = IMG_I(sensor_type)[tid]; q_id = IMG_I(sensor_objid)[tid]; q_adr = IMG_I(sensor_adr)[tid];
      q_bits = IMG_I(sensor_intprm)[3 * tid]; q_red = IMG_I(sensor_intprm)[3 * tid + 1];
      q_nslot = IMG_I(sensor_intprm)[3 * tid + 2]; q_ot = IMG_I(sensor_objtype)[tid];
      q_rt = IMG_I(sensor_reftype)[tid]; q_rid = IMG_I(sensor_refid)[tid]; q_dim = IMG_I(sensor_dim)[tid];
    }
    auto sq = [&](int v, const int* p, int s) -> int { return s < NT ? __builtin_amdgcn_readlane(v, s) : p[s]; };
#elif MJH_SENS_PRELOAD == 2
    // [type | objtype << 8 | reftype << 14 | bits << 20 | reduce << 27], adr,
    // [(objid + 1) | (refid + 1) << 16], [nslot | dim << 16] (field ranges checked by
    // the compiler, spec/compiler.py)
    int q_a = -1, q_b = 0, q_c = 0, q_d = 0;
    if (tid < Z.nsensor) {
      q_a = IMG_I(sensor_type)[tid] | IMG_I(sensor_objtype)[tid] << 8 | IMG_I(sensor_reftype)[tid] << 14 |
            IMG_I(sensor_intprm)[3 * tid] << 20 | IMG_I(sensor_intprm)[3 * tid + 1] << 27;
      q_b = IMG_I(sensor_adr)[tid];
      q_c = (IMG_I(sensor_objid)[tid] + 1) | (IMG_I(sensor_refid)[tid] + 1) << 16;
      q_d = IMG_I(sensor_intprm)[3 * tid + 2] | IMG_I(sensor_dim)[tid] << 16;
    }
#endif
    // geom g (body gb, subtree mask tm) matches object (ty, oid)
    auto om_match = [](int ty, int oid, int g, int gb, unsigned long long tm) -> bool {
      if (oid < 0) return true;
      if (ty == 5) return g == oid;
      if (ty == 1) return gb == oid;
      if (ty == 2) return oid == 0 || ((tm >> oid) & 1ull);
      return false;
    };
    // match / flip ballots of contact sensor s at pmb[2 s], pmb[2 s + 1] (contacts in
    // lanes: ncon <= 64; sensor metadata in lanes: nsensor <= 64)
    unsigned long long* const pmb = reinterpret_cast<unsigned long long*>(ash);
    bool pm = MJH_SENS_PREMATCH && MJH_SENS_PRELOAD == 2 && !MJH_SENS_OMREG && creg && Z.nsensor <= NT &&
              4 * Z.nsensor <= acap + 4;
#if MJH_SENS_PRELOAD == 2
    pm = pm && __ballot((q_a & 255) == 40) != 0ull;  // a contact sensor at all (q_a is -1 past nsensor)
    if (pm) {
      int g1 = 0, g2 = 0, b1 = 0, b2 = 0;
      unsigned long long t1 = 0ull, t2 = 0ull;
      const bool cl = tid < ncon;
      if (cl) {
        g1 = con_geom[2 * tid];
        g2 = con_geom[2 * tid + 1];
        b1 = IMG_I(geom_bodyid)[g1];
        b2 = IMG_I(geom_bodyid)[g2];
        t1 = (unsigned long long)IMG_L(body_treemask)[b1];
        t2 = (unsigned long long)IMG_L(body_treemask)[b2];
      }
      for (int s = 0; s < Z.nsensor; s++) {
        const int qa = __builtin_amdgcn_readlane(q_a, s);
        if ((qa & 255) != 40) continue;
        const int qc = __builtin_amdgcn_readlane(q_c, s);
        const int otype = (qa >> 8) & 63, rtype = (qa >> 14) & 63, id = (qc & 0xffff) - 1, rid = (qc >> 16) - 1;
        bool match = false, flip = false;
        if (cl) {
          if (om_match(otype, id, g1, b1, t1) && om_match(rtype, rid, g2, b2, t2)) match = true;
          else if (om_match(otype, id, g2, b2, t2) && om_match(rtype, rid, g1, b1, t1)) { match = true; flip = true; }
        }
        const unsigned long long mb = __ballot(match), fb = __ballot(flip);
        if (tid == 0) {
          pmb[2 * s] = mb;
          pmb[2 * s + 1] = fb;
        }
      }
      wsync();
    }
#endif
    auto contact_force = [&](int ci, float (&F)[6]) {
#pragma unroll
      for (int k = 0; k < 6; k++) F[k] = 0.f;
      const int r0 = con_efcadr[ci];
      if (r0 >= 0) {
        const int cdm = con_dim[ci];
        if (cdm == 1) {
          F[0] = efc_force[r0];
        } else if (ELL) {  // elliptic: the rows are the frame components
          for (int k = 0; k < cdm && k < 6; k++) F[k] = efc_force[r0 + k];
        } else {
          for (int e = 0; e < 2 * (cdm - 1); e++) F[0] += efc_force[r0 + e];
          for (int k = 1; k < cdm && k < 6; k++) F[k] = con_fric[5 * ci + k - 1] * (efc_force[r0 + 2 * k - 2] - efc_force[r0 + 2 * k - 1]);
        }
      }
    };
    // the previous contact sensor's match parameters and count: mjlab declares
    // one sensor per (primary, field), so consecutive sensors (found, force of
    // the same foot) repeat the same scan; the kept matches are still in sx
    int p_ot = -9, p_id = -9, p_rt = -9, p_rid = -9, p_cnt = 0;
    for (int s = 0; s < Z.nsensor; s++) {
#if MJH_SENS_PRELOAD == 1
      const int type = sq(q_type, IMG_I(sensor_type), s), id = sq(q_id, IMG_I(sensor_objid), s);
      const int adr = sq(q_adr, IMG_I(sensor_adr), s);
#elif MJH_SENS_PRELOAD == 2
      const bool qr = s < NT;
      const int qa = qr ? __builtin_amdgcn_readlane(q_a, s) : 0, qc = qr ? __builtin_amdgcn_readlane(q_c, s) : 0;
      const int type = qr ? (qa & 255) : IMG_I(sensor_type)[s];
      const int id = qr ? (qc & 0xffff) - 1 : IMG_I(sensor_objid)[s];
      const int adr = qr ? __builtin_amdgcn_readlane(q_b, s) : IMG_I(sensor_adr)[s];
#else
      const int type = IMG_I(sensor_type)[s], id = IMG_I(sensor_objid)[s], adr = IMG_I(sensor_adr)[s];
#endif
      if (type == 40) {
        // contact sensor (MuJoCo mjSENS_CONTACT with mjlab's intprm encoding,
        // contact_sensor.py:472-496): matches in contact order, capped at
        // min(maxmatch, 64); then one lane per kept match.
        const int* ip = IMG_I(sensor_intprm);
#if MJH_SENS_PRELOAD == 1
        const int bits = s < NT ? __builtin_amdgcn_readlane(q_bits, s) : ip[3 * s];
        const int reduce = s < NT ? __builtin_amdgcn_readlane(q_red, s) : ip[3 * s + 1];
        const int nslot = s < NT ? __builtin_amdgcn_readlane(q_nslot, s) : ip[3 * s + 2];
        const int otype = sq(q_ot, IMG_I(sensor_objtype), s), rtype = sq(q_rt, IMG_I(sensor_reftype), s);
        const int rid = sq(q_rid, IMG_I(sensor_refid), s);
        const int dim = sq(q_dim, IMG_I(sensor_dim), s);
#elif MJH_SENS_PRELOAD == 2
        const int qd = qr ? __builtin_amdgcn_readlane(q_d, s) : 0;
        const int bits = qr ? (qa >> 20) & 127 : ip[3 * s];
        const int reduce = qr ? (qa >> 27) & 7 : ip[3 * s + 1];
        const int nslot = qr ? (qd & 0xffff) : ip[3 * s + 2];
        const int otype = qr ? (qa >> 8) & 63 : IMG_I(sensor_objtype)[s], rtype = qr ? (qa >> 14) & 63 : IMG_I(sensor_reftype)[s];
        const int rid = qr ? (qc >> 16) - 1 : IMG_I(sensor_refid)[s];
        const int dim = qr ? (qd >> 16) : IMG_I(sensor_dim)[s];
#else
        const int bits = ip[3 * s], reduce = ip[3 * s + 1], nslot = ip[3 * s + 2];
        const int otype = IMG_I(sensor_objtype)[s], rtype = IMG_I(sensor_reftype)[s], rid = IMG_I(sensor_refid)[s];
        const int dim = IMG_I(sensor_dim)[s];
#endif
        const int cap = min(m.contact_sensor_maxmatch, 64);
        // kept matches in the solver's (now dead) LDS row-index array when it is
        // large enough (always for the benchmark models), else in global scratch.
        // The record is zeroed where it is written (below), so no store precedes
        // this sensor's scratch loads.
        int* const sx = acap + 4 >= 64 ? arow : sidx;
        // the match list lives in LDS for the benchmark models (then only LDS
        // ordering matters between its writes and reads: no wait for the
        // sensordata stores in flight), else in global scratch
        const bool sx_lds = MJH_SENS_LSYNC && (acap + 4 >= 64 ? (!BIG && !Rg::arow) : !Rg::sidx);
        auto sx_fence = [&]() {
          if (sx_lds) lsync(); else wsync();
        };
        // geom g (body gb, subtree mask tm) matches object (ty, oid)
        auto om_b = [&](int ty, int oid, int g, int gb, unsigned long long tm) -> bool {
          if (oid < 0) return true;
          if (ty == 5) return g == oid;
          if (ty == 1) return gb == oid;
          if (ty == 2) return oid == 0 || ((tm >> oid) & 1ull);
          return false;
        };
        auto om = [&](int ty, int oid, int g) -> bool {
          const int gb = IMG_I(geom_bodyid)[g];
          return om_b(ty, oid, g, gb, (unsigned long long)IMG_L(body_treemask)[gb]);
        };
        if (creg && !cloaded) {
          cloaded = true;
#pragma unroll
          for (int k = 0; k < 6; k++) cF[k] = 0.f;
#pragma unroll
          for (int k = 0; k < 9; k++) cfr[k] = 0.f;
          cps[0] = cps[1] = cps[2] = 0.f;
          if (tid < ncon) {
            cg1 = con_geom[2 * tid];
            cg2 = con_geom[2 * tid + 1];
#pragma unroll
            for (int k = 0; k < 9; k++) cfr[k] = con_frame[9 * tid + k];
#pragma unroll
            for (int k = 0; k < 3; k++) cps[k] = con_pos[3 * tid + k];
            cds = con_dist[tid];
            contact_force(tid, cF);
            if (MJH_SENS_OMREG) {
              cb1 = IMG_I(geom_bodyid)[cg1];
              cb2 = IMG_I(geom_bodyid)[cg2];
              ct1 = (unsigned long long)IMG_L(body_treemask)[cb1];
              ct2 = (unsigned long long)IMG_L(body_treemask)[cb2];
            }
          }
        }
        int cnt = 0;
        if (otype == p_ot && id == p_id && rtype == p_rt && rid == p_rid) {
          cnt = p_cnt;  // same matches as the previous contact sensor (sx unchanged)
        } else if (pm) {
          // the pre-pass's ballots: the same list, in contact order, as the scan below
          const unsigned long long mb = pmb[2 * s], fb = pmb[2 * s + 1];
          cnt = __popcll(mb);
          if ((mb >> tid) & 1ull) {
            const int off = __popcll(mb & ((1ull << tid) - 1ull));
            if (off < cap) sx[off] = ((fb >> tid) & 1ull) ? ~tid : tid;
          }
          sx_fence();
          p_ot = otype; p_id = id; p_rt = rtype; p_rid = rid; p_cnt = cnt;
        } else {
          for (int base = 0; base < ncon; base += NT) {
            const int ci = base + tid;
            int match = 0, flip = 0;
            if (MJH_SENS_OMREG && ci < ncon && creg) {  // bodies and subtree masks in registers
              if (om_b(otype, id, cg1, cb1, ct1) && om_b(rtype, rid, cg2, cb2, ct2)) match = 1;
              else if (om_b(otype, id, cg2, cb2, ct2) && om_b(rtype, rid, cg1, cb1, ct1)) { match = 1; flip = 1; }
            } else if (ci < ncon) {
              const int g1 = con_geom[2 * ci], g2 = con_geom[2 * ci + 1];
              if (om(otype, id, g1) && om(rtype, rid, g2)) match = 1;
              else if (om(otype, id, g2) && om(rtype, rid, g1)) { match = 1; flip = 1; }
            }
            int total;
            const int off = bscan<NT>(match, &total, redi);
            if (match && cnt + off < cap) sx[cnt + off] = flip ? ~ci : ci;
            cnt += total;
          }
          sx_fence();
          p_ot = otype; p_id = id; p_rt = rtype; p_rid = rid; p_cnt = cnt;
        }
        const int nm = min(cnt, cap);
        if (nm == 0) {
          for (int k = tid; k < dim; k += NT) sd[adr + k] = 0.f;
          continue;
        }
        if (bits == 1) {
          // found only: the match count in the first min(nm, nslot) slots (one
          // record for netforce), zeros after — what the general path writes
          for (int k = tid; k < dim; k += NT) sd[adr + k] = (reduce == 3 ? k == 0 : k < nm) ? (float)nm : 0.f;
          sx_fence();  // only the match list needs ordering (the sensordata stores need none)
          continue;
        }
        // lane k < nm: match k. F = contact force/torque in the contact frame
        // (mj_contactForce for pyramidal cones), Fw/Tw = on the primary, world frame
        const bool own = tid < nm;
        const int code = own ? sx[tid] : 0;
        const int ci = code < 0 ? ~code : code;
        const float sgn = code < 0 ? 1.f : -1.f;
        float F[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, Fw[3] = {0.f, 0.f, 0.f}, Tw[3] = {0.f, 0.f, 0.f};
        float cpos[3] = {0.f, 0.f, 0.f}, cdist = 0.f, fr[9];
        if (creg) {
          const int src = own ? ci : 0;  // every lane takes part in the permutes
#pragma unroll
          for (int k = 0; k < 6; k++) F[k] = shfl(cF[k], src);
#pragma unroll
          for (int k = 0; k < 9; k++) fr[k] = shfl(cfr[k], src);
#pragma unroll
          for (int k = 0; k < 3; k++) cpos[k] = shfl(cps[k], src);
          cdist = shfl(cds, src);
        } else if (own) {
          contact_force(ci, F);
#pragma unroll
          for (int k = 0; k < 9; k++) fr[k] = con_frame[9 * ci + k];
#pragma unroll
          for (int k = 0; k < 3; k++) cpos[k] = con_pos[3 * ci + k];
          cdist = con_dist[ci];
        }
        if (own) {
          for (int a = 0; a < 3; a++) {
            Fw[a] = sgn * (F[0] * fr[a] + F[1] * fr[3 + a] + F[2] * fr[6 + a]);
            Tw[a] = sgn * (F[3] * fr[a] + F[4] * fr[3 + a] + F[5] * fr[6 + a]);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 6; k++) F[k] = 0.f;
          cpos[0] = cpos[1] = cpos[2] = 0.f;
          cdist = 0.f;
        }
        const float found = (float)nm;
        if (reduce == 3) {
          // netforce: net wrench at the force-weighted centroid (weights |Fw|)
          const float fn = sqrtf(dot3(Fw, Fw));
          float nx = Fw[0], ny = Fw[1], nz = Fw[2], cx = fn * cpos[0], cy = fn * cpos[1], cz = fn * cpos[2], ws = fn, z = 0.f;
          bsum2<NT>(nx, ny, red);
          bsum2<NT>(nz, ws, red);
          bsum2<NT>(cx, cy, red);
          bsum2<NT>(cz, z, red);
          float dmin = own ? cdist : 3.0e38f;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) dmin = fminf(dmin, __shfl_xor(dmin, o, 64));
          float cen[3];
          if (ws > MJH_MINVAL) { cen[0] = cx / ws; cen[1] = cy / ws; cen[2] = cz / ws; }
          else { cen[0] = rl(cpos[0], 0); cen[1] = rl(cpos[1], 0); cen[2] = rl(cpos[2], 0); }
          float rr[3] = {cpos[0] - cen[0], cpos[1] - cen[1], cpos[2] - cen[2]}, t[3];
          cross3(t, rr, Fw);
          float tx = own ? t[0] + Tw[0] : 0.f, ty = own ? t[1] + Tw[1] : 0.f, tz = own ? t[2] + Tw[2] : 0.f, z2 = 0.f;
          bsum2<NT>(tx, ty, red);
          bsum2<NT>(tz, z2, red);
          if (tid == 0) {
            float* o = sd + adr;
            int q = 0;
            if (bits & 1) o[q++] = found;
            if (bits & 2) { o[q++] = nx; o[q++] = ny; o[q++] = nz; }
            if (bits & 4) { o[q++] = tx; o[q++] = ty; o[q++] = tz; }
            if (bits & 8) o[q++] = dmin;
            if (bits & 16) { o[q++] = cen[0]; o[q++] = cen[1]; o[q++] = cen[2]; }
            if (bits & 32) { o[q++] = 0.f; o[q++] = 0.f; o[q++] = 0.f; }
            if (bits & 64) { o[q++] = 0.f; o[q++] = 0.f; o[q++] = 0.f; }
          }
          sx_fence();  // only the match list needs ordering (the sensordata stores need none)
          continue;
        }
        // none: contact order; mindist: dist ascending; maxforce: |F| descending
        // (stable: ties keep contact order)
        int rank = tid;
        if (reduce == 1 || reduce == 2) {
          const float key = reduce == 1 ? cdist : -sqrtf(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]);
          rank = 0;
          for (int j = 0; j < nm; j++) {
            const float kj = rl(key, j);
            rank += (kj < key || (kj == key && j < tid)) ? 1 : 0;
          }
        }
        if (own && rank < nslot) {
          float* o = sd + adr + rank * (dim / nslot);
          const float sg = code < 0 ? -1.f : 1.f;  // normal primary -> secondary
          int q = 0;
          if (bits & 1) o[q++] = found;
          if (bits & 2) { o[q++] = F[0]; o[q++] = F[1]; o[q++] = F[2]; }
          if (bits & 4) { o[q++] = F[3]; o[q++] = F[4]; o[q++] = F[5]; }
          if (bits & 8) o[q++] = cdist;
          if (bits & 16) { o[q++] = cpos[0]; o[q++] = cpos[1]; o[q++] = cpos[2]; }
          if (bits & 32) { o[q++] = sg * fr[0]; o[q++] = sg * fr[1]; o[q++] = sg * fr[2]; }
          if (bits & 64) { o[q++] = sg * fr[3]; o[q++] = sg * fr[4]; o[q++] = sg * fr[5]; }
        }
        for (int k = nm * (dim / nslot) + tid; k < dim; k += NT) sd[adr + k] = 0.f;  // slots without a match
        sx_fence();  // only the match list needs ordering (the sensordata stores need none)
        continue;
      }
#ifndef MJH_NO_EXT
      if ((Z.sensor_ext_mask & kExtEnergy) && (type == 48 || type == 49)) {  // compile-time 0 in the benchmark models' instances
        // e_potential (mj_energyPos: gravity over bodies + joint springs) /
        // e_kinetic (mj_energyVel: qvel' M qvel / 2, M rows from the factor pass)
        float e = 0.f, z = 0.f;
        if (type == 48) {
          for (int b = 1 + tid; b < nb; b += NT)
            e -= cinert[10 * b + 9] * (m.gravity_x * xipos[3 * b] + m.gravity_y * xipos[3 * b + 1] + m.gravity_z * xipos[3 * b + 2]);
          for (int j = tid; j < Z.njnt; j += NT) {
            const float k = jnt_stiffness[j];
            const int t = IMG_I(jnt_type)[j];
            if (k == 0.f || t == 0) continue;
            const int qa = IMG_I(jnt_qposadr)[j];
            if (t == 1) {
              float dif[3];
              sub_quat(dif, qpos + qa, IMG_F(qpos_spring) + qa);
              e += 0.5f * k * dot3(dif, dif);
            } else {
              const float dq = qpos[qa] - IMG_F(qpos_spring)[qa];
              e += 0.5f * k * dq * dq;
            }
          }
        } else {
          for (int i = tid; i < nv; i += NT) {
            float r = 0.f;
            for (int j = 0; j < nv; j++) r += Mm[i * ldm + j] * qvel[j];
            e += 0.5f * qvel[i] * r;
          }
        }
        bsum2<NT>(e, z, red);
        if (tid == 0) sd[adr] = e;
        continue;
      }
#endif
      if (type != 35 && type != 36) continue;
      // subtree linvel / angmom: lanes over bodies, wave reductions
      const unsigned long long* tmask = (const unsigned long long*)IMG_L(body_treemask);
      auto in_tree = [&](int b) { return id == 0 || ((tmask[b] >> id) & 1ull); };
      float msum = 0.f, l0 = 0.f, l1 = 0.f, l2 = 0.f;
      for (int b = 1 + tid; b < nb; b += NT) {
        if (!in_tree(b)) continue;
        const float bm = cinert[10 * b + 9];
        const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
        const float* v = cvel + 6 * b;
        float dif[3] = {xipos[3 * b] - c[0], xipos[3 * b + 1] - c[1], xipos[3 * b + 2] - c[2]}, t[3];
        cross3(t, dif, v);
        msum += bm;
        l0 += bm * (v[3] - t[0]); l1 += bm * (v[4] - t[1]); l2 += bm * (v[5] - t[2]);
      }
      bsum2<NT>(msum, l0, red);
      bsum2<NT>(l1, l2, red);
      float vc[3] = {0.f, 0.f, 0.f};
      if (msum > MJH_MINVAL) { vc[0] = l0 / msum; vc[1] = l1 / msum; vc[2] = l2 / msum; }
      float* out = sd + adr;
      float o3[3] = {vc[0], vc[1], vc[2]};
      if (type == 36) {
        float L0 = 0.f, L1 = 0.f, L2 = 0.f;
        const float* sc = subtree_com + 3 * id;
        for (int b = 1 + tid; b < nb; b += NT) {
          if (!in_tree(b)) continue;
          const float bm = cinert[10 * b + 9];
          const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
          const float* v = cvel + 6 * b;
          float dd[3] = {xipos[3 * b] - c[0], xipos[3 * b + 1] - c[1], xipos[3 * b + 2] - c[2]}, t[3];
          cross3(t, dd, v);
          float vb[3] = {v[3] - t[0], v[4] - t[1], v[5] - t[2]};
          const float* ci = cinert + 10 * b;
          const float dsq = dot3(dd, dd);
          float I[9] = {ci[0] - bm * (dsq - dd[0] * dd[0]), ci[3] + bm * dd[0] * dd[1], ci[4] + bm * dd[0] * dd[2],
                        ci[3] + bm * dd[0] * dd[1], ci[1] - bm * (dsq - dd[1] * dd[1]), ci[5] + bm * dd[1] * dd[2],
                        ci[4] + bm * dd[0] * dd[2], ci[5] + bm * dd[1] * dd[2], ci[2] - bm * (dsq - dd[2] * dd[2])};
          float Iw[3], dx[3], dv[3];
          mat_vec(Iw, I, v);
          for (int k = 0; k < 3; k++) { dx[k] = xipos[3 * b + k] - sc[k]; dv[k] = (vb[k] - vc[k]) * bm; }
          cross3(t, dx, dv);
          L0 += Iw[0] + t[0]; L1 += Iw[1] + t[1]; L2 += Iw[2] + t[2];
        }
        float z = 0.f;
        bsum2<NT>(L0, L1, red);
        bsum2<NT>(L2, z, red);
        o3[0] = L0; o3[1] = L1; o3[2] = L2;
      }
      if (tid == 0) {
        const float cut = IMG_F(sensor_cutoff)[s];
        for (int k = 0; k < 3; k++) out[k] = cut > 0.f ? clampf(o3[k], -cut, cut) : o3[k];
      }
    }
#ifndef MJH_NO_FT
    // force / torque sensors (mj_sensorAcc), in a pass of their own so that no
    // state of theirs is live in the loop above
    for (int s = 0; s < ((Z.sensor_ext_mask & kExtForce) ? Z.nsensor : 0); s++) {
      const int type = IMG_I(sensor_type)[s];
      if (type != 4 && type != 5) continue;
      const int id = IMG_I(sensor_objid)[s];
      force_torque_sensor(tid, nb, ncon, type, IMG_I(site_bodyid)[id], sxpos + 3 * id, sxmat + 9 * id, IMG_F(sensor_cutoff)[s],
                          cinert, cacc, cvel, xipos, subtree_com, DP(xfrc_applied) + W * nb * 6, IMG_I(body_rootid),
                          IMG_I(geom_bodyid), con_frame, con_pos, con_geom, con_efcadr, con_dim, con_fric, efc_force, ELL,
                          r_tmk, sd + IMG_I(sensor_adr)[s]);
    }
#endif
    // a sensor object's frame (mj_sensorPos): 1 body (inertial frame), 2 xbody,
    // 5 geom (from its body's frame, as the geom pass computes it), 6 site; b:
    // the body it moves with
    auto obj_frame = [&](int ot, int oid, float (&p)[3], float (&R)[9], int& b) {
      if (ot == 5) {
        b = IMG_I(geom_bodyid)[oid];
        float t[3], GR[9];
        mat_vec(t, xmat + 9 * b, geom_pos + 3 * oid);
        for (int k = 0; k < 3; k++) p[k] = xpos[3 * b + k] + t[k];
        quat2mat(GR, geom_quat + 4 * oid);
        mat_mul(R, xmat + 9 * b, GR);
        return;
      }
      const float* sp = ot == 1 ? xipos + 3 * oid : (ot == 2 ? xpos + 3 * oid : sxpos + 3 * oid);
      const float* sR = ot == 1 ? ximat + 9 * oid : (ot == 2 ? xmat + 9 * oid : sxmat + 9 * oid);
      b = ot == 1 || ot == 2 ? oid : IMG_I(site_bodyid)[oid];
      for (int k = 0; k < 3; k++) p[k] = sp[k];
      for (int k = 0; k < 9; k++) R[k] = sR[k];
    };
    // its orientation: xbody copies xquat, body composes the inertial frame's
    // quaternion, geom / site convert their matrix
    auto obj_quat = [&](int ot, int oid, float (&q)[4]) {
      if (ot == 2) {
        for (int k = 0; k < 4; k++) q[k] = xquat[4 * oid + k];
      } else if (ot == 1) {
        float a[4] = {xquat[4 * oid], xquat[4 * oid + 1], xquat[4 * oid + 2], xquat[4 * oid + 3]};
        quat_mul(q, a, body_iquat + 4 * oid);
      } else {
        float p[3], R[9];
        int b;
        obj_frame(ot, oid, p, R, b);
        mat2quat(q, R);
      }
    };
    // 6D world velocity [angular; linear at point p] of body b (mj_objectVelocity, flg_local 0)
    auto obj_vel = [&](const float (&p)[3], int b, float (&v)[6]) {
      const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
      const float* cv = cvel + 6 * b;
      const float dif[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
      float t[3];
      cross3(t, dif, cv);
      v[0] = cv[0]; v[1] = cv[1]; v[2] = cv[2];
      v[3] = cv[3] - t[0]; v[4] = cv[4] - t[1]; v[5] = cv[5] - t[2];
    };
    // the sensor types outside the benchmark tasks' set, by group (Sizes::sensor_ext_mask: an
    // instance specialised for a model compiles in only the groups the model has)
    auto ext_sensor = [&](int s, int type, int id, float* out) {
      switch (type) {
        case 30:
        case 41:
        case 42:
        case 43: {  // framepos / frame{x,y,z}axis, optionally in the ref frame (mj_sensorPos)
          if (!(Z.sensor_ext_mask & kExtFramePos)) break;
          float p[3], R[9], pr[3], Rr[9], v[3];
          int b, br;
          obj_frame(IMG_I(sensor_objtype)[s], id, p, R, b);
          if (type == 30) { v[0] = p[0]; v[1] = p[1]; v[2] = p[2]; }
          else { const int c = type - 41; v[0] = R[c]; v[1] = R[3 + c]; v[2] = R[6 + c]; }
          const int rid = IMG_I(sensor_refid)[s];
          if (rid >= 0) {
            obj_frame(IMG_I(sensor_reftype)[s], rid, pr, Rr, br);
            if (type == 30) { v[0] -= pr[0]; v[1] -= pr[1]; v[2] -= pr[2]; }
            matT_vec(v, Rr, v);
          }
          out[0] = v[0]; out[1] = v[1]; out[2] = v[2];
          break;
        }
        case 31: {  // framequat, relative to the ref frame when one is given: conj(q_ref) * q
          if (!(Z.sensor_ext_mask & kExtFrameQuat)) break;
          float q[4];
          obj_quat(IMG_I(sensor_objtype)[s], id, q);
          const int rid = IMG_I(sensor_refid)[s];
          if (rid >= 0) {
            float qr[4];
            obj_quat(IMG_I(sensor_reftype)[s], rid, qr);
            qr[1] = -qr[1]; qr[2] = -qr[2]; qr[3] = -qr[3];
            quat_mul(q, qr, q);
          }
          out[0] = q[0]; out[1] = q[1]; out[2] = q[2]; out[3] = q[3];
          break;
        }
        case 44:
        case 45: {  // framelinvel / frameangvel (mj_sensorVel): world frame, or relative to the ref frame and in it
          if (!(Z.sensor_ext_mask & kExtFrameVel)) break;
          float p[3], R[9], v[6];
          int b;
          obj_frame(IMG_I(sensor_objtype)[s], id, p, R, b);
          obj_vel(p, b, v);
          const int rid = IMG_I(sensor_refid)[s];
          float r[3];
          if (rid < 0) {
            const float* o = type == 44 ? v + 3 : v;
            r[0] = o[0]; r[1] = o[1]; r[2] = o[2];
          } else {
            float pr[3], Rr[9], vr[6], t[3];
            int br;
            obj_frame(IMG_I(sensor_reftype)[s], rid, pr, Rr, br);
            obj_vel(pr, br, vr);
            if (type == 44) {
              const float dp[3] = {p[0] - pr[0], p[1] - pr[1], p[2] - pr[2]};
              cross3(t, vr, dp);
              r[0] = v[3] - vr[3] - t[0]; r[1] = v[4] - vr[4] - t[1]; r[2] = v[5] - vr[5] - t[2];
            } else {
              r[0] = v[0] - vr[0]; r[1] = v[1] - vr[1]; r[2] = v[2] - vr[2];
            }
            matT_vec(r, Rr, r);
          }
          out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
          break;
        }
        case 46:
        case 47: {  // framelinacc / frameangacc (mj_objectAcceleration, world frame): cacc at the frame origin + w x v
          if (!(Z.sensor_ext_mask & kExtFrameAcc)) break;
          float p[3], R[9];
          int b;
          obj_frame(IMG_I(sensor_objtype)[s], id, p, R, b);
          const float* a = cacc + 6 * b;
          if (type == 47) { out[0] = a[0]; out[1] = a[1]; out[2] = a[2]; break; }
          const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
          const float dif[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
          float v[6], t[3], al[3];
          obj_vel(p, b, v);
          cross3(t, dif, a);
          al[0] = a[3] - t[0]; al[1] = a[4] - t[1]; al[2] = a[5] - t[2];
          cross3(t, v, v + 3);
          out[0] = al[0] + t[0]; out[1] = al[1] + t[1]; out[2] = al[2] + t[2];
          break;
        }
        case 20:
        case 21:
        case 22: {  // jointlimitpos / vel / frc: the joint's limit row (efc_pos - margin, J qvel, force); 0 if inactive
          if (!(Z.sensor_ext_mask & kExtLimit)) break;
          float val = 0.f;
          const int nr = min(nefc, Lo.rcap);
          for (int r = 0; r < nr; r++) {
            if (efc_type[r] != MJH_CNSTR_LIMIT_JOINT || efc_id[r] != id) continue;
            val = type == 20 ? efc_pos[r] - IMG_F(jnt_margin)[id] : (type == 21 ? rowdot_u<NVP>(J + r * ldj, qvel, nv) : efc_force[r]);
            break;
          }
          out[0] = val;
          break;
        }
        case 13:  // actuatorpos / actuatorvel: gear * joint coordinate (joint transmission)
        case 14: {
          if (!(Z.sensor_ext_mask & kExtActuator)) break;
          const int j = IMG_I(actuator_trnid)[id];
          out[0] = IMG_F(actuator_gear)[id] * (type == 13 ? qpos[IMG_I(jnt_qposadr)[j]] : qvel[IMG_I(jnt_dofadr)[j]]);
          break;
        }
        case 15: if (Z.sensor_ext_mask & kExtActuator) out[0] = act_force[id]; break;
        case 16: if (Z.sensor_ext_mask & kExtActuator) out[0] = qfrc_act[IMG_I(jnt_dofadr)[id]]; break;
        case 18: {  // ballquat: the normalised joint quaternion
          if (!(Z.sensor_ext_mask & kExtBall)) break;
          float q[4];
          const float* qp = qpos + IMG_I(jnt_qposadr)[id];
          q[0] = qp[0]; q[1] = qp[1]; q[2] = qp[2]; q[3] = qp[3];
          quat_normalize(q);
          out[0] = q[0]; out[1] = q[1]; out[2] = q[2]; out[3] = q[3];
          break;
        }
        case 19: {
          if (!(Z.sensor_ext_mask & kExtBall)) break;
          const float* qv = qvel + IMG_I(jnt_dofadr)[id];
          out[0] = qv[0]; out[1] = qv[1]; out[2] = qv[2];
          break;
        }
        case 50: if (Z.sensor_ext_mask & kExtClock) out[0] = DP(time)[W]; break;
        case 7: {  // rangefinder (mj_ray along the site's z axis; not the site body's geoms, not rgba alpha 0)
          if (!(Z.sensor_ext_mask & kExtRange)) break;
          const float* R = sxmat + 9 * id;
          const float vec[3] = {R[2], R[5], R[8]};
          const float* rgba = WFIELD(geom_rgba);
          const int bex = IMG_I(site_bodyid)[id];
          float best = -1.f;
          for (int g = 0; g < Z.ngeom; g++) {
            if (IMG_I(geom_bodyid)[g] == bex || rgba[4 * g + 3] == 0.f) continue;
            float gp[3], gR[9];
            int gb;
            obj_frame(5, g, gp, gR, gb);
            const float dd = ray_geom(IMG_I(geom_type)[g], IMG_F(geom_size) + 3 * g, gp, gR, sxpos + 3 * id, vec);
            if (dd >= 0.f && (best < 0.f || dd < best)) best = dd;
          }
          out[0] = best;
          break;
        }
        case 6: {  // magnetometer: the global field in the site frame
          if (!(Z.sensor_ext_mask & kExtMag)) break;
          const float mg[3] = {m.magnetic_x, m.magnetic_y, m.magnetic_z};
          float r[3];
          matT_vec(r, sxmat + 9 * id, mg);
          out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
          break;
        }
        default:
          break;
      }
    };
    PROF(11);
    // remaining sensors are independent and cheap: one lane each
    for (int s = tid; s < Z.nsensor; s += NT) {
      const int type = IMG_I(sensor_type)[s], id = IMG_I(sensor_objid)[s], adr = IMG_I(sensor_adr)[s];
      if (type == 40 || type == 35 || type == 36 || type == 48 || type == 49 || type == 4 || type == 5) continue;
      float* out = sd + adr;
      switch (type) {
        case 3: {  // gyro
          const int b = IMG_I(site_bodyid)[id];
          float r[3];
          matT_vec(r, sxmat + 9 * id, cvel + 6 * b);
          out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
          break;
        }
        case 2:
        case 1: {  // velocimeter / accelerometer
          const int b = IMG_I(site_bodyid)[id];
          const float* c = subtree_com + 3 * IMG_I(body_rootid)[b];
          const float* sp = sxpos + 3 * id;
          float dif[3] = {sp[0] - c[0], sp[1] - c[1], sp[2] - c[2]}, t[3], lin[3], r[3];
          const float* v = cvel + 6 * b;
          cross3(t, dif, v);
          lin[0] = v[3] - t[0]; lin[1] = v[4] - t[1]; lin[2] = v[5] - t[2];
          matT_vec(r, sxmat + 9 * id, lin);
          if (type == 2) {
            out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
          } else {
            const float* a = cacc + 6 * b;
            float al[3], ar[3], wl[3], cor[3];
            cross3(t, dif, a);
            al[0] = a[3] - t[0]; al[1] = a[4] - t[1]; al[2] = a[5] - t[2];
            matT_vec(ar, sxmat + 9 * id, al);
            matT_vec(wl, sxmat + 9 * id, v);
            cross3(cor, wl, r);
            out[0] = ar[0] + cor[0]; out[1] = ar[1] + cor[1]; out[2] = ar[2] + cor[2];
          }
          break;
        }
        case 9: out[0] = qpos[IMG_I(jnt_qposadr)[id]]; break;
        case 10: out[0] = qvel[IMG_I(jnt_dofadr)[id]]; break;
        case 34: out[0] = subtree_com[3 * id]; out[1] = subtree_com[3 * id + 1]; out[2] = subtree_com[3 * id + 2]; break;
        default:
          if (Z.sensor_ext_mask != 0) ext_sensor(s, type, id, out);  // compile-time 0 in the benchmark models' instances
          break;
      }
      const float cut = IMG_F(sensor_cutoff)[s];
      if (cut > 0.f && type == 7)  // rangefinder (mjDATATYPE_POSITIVE): clipped above only, a miss stays -1
        out[0] = fminf(out[0], cut);
      else if (cut > 0.f && type != 31 && type != 18 && (type < 41 || type > 43))  // quaternions and unit axes are not clipped
        for (int k = 0; k < IMG_I(sensor_dim)[s]; k++) out[k] = clampf(out[k], -cut, cut);
    }
  }
  wsync();

  // ---------------------------------------------------------------- forward outputs
  PROF(7);
  // Each lane loads everything it copies before its first store: the data
  // arrays may alias the scratch as far as the compiler knows, and a load
  // issued after a store waits for the store too (one memory latency per
  // array otherwise). Lane = body / joint / site / dof / contact / row.
  if (!kOutDirect && tid < nb) {
    const int b = tid;
    float v[43];
#pragma unroll
    for (int k = 0; k < 3; k++) { v[k] = xpos[3 * b + k]; v[3 + k] = xipos[3 * b + k]; v[6 + k] = subtree_com[3 * b + k]; }
#pragma unroll
    for (int k = 0; k < 4; k++) v[9 + k] = xquat[4 * b + k];
#pragma unroll
    for (int k = 0; k < 9; k++) { v[13 + k] = xmat[9 * b + k]; v[22 + k] = ximat[9 * b + k]; }
#pragma unroll
    for (int k = 0; k < 6; k++) { v[31 + k] = cvel[6 * b + k]; v[37 + k] = cacc[6 * b + k]; }
    const long long o = (long long)W * nb + b;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      DP(xpos)[3 * o + k] = v[k];
      DP(xipos)[3 * o + k] = v[3 + k];
      DP(subtree_com)[3 * o + k] = v[6 + k];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) DP(xquat)[4 * o + k] = v[9 + k];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      DP(xmat)[9 * o + k] = v[13 + k];
      DP(ximat)[9 * o + k] = v[22 + k];
    }
#pragma unroll
    for (int k = 0; k < 6; k++) {
      DP(cvel)[6 * o + k] = v[31 + k];
      DP(cacc)[6 * o + k] = v[37 + k];
    }
  }
  {
    float vj[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, vs[12], vd[8];
    const bool jl = tid < nj, sl = tid < Z.nsite, dl = tid < nv;  // nj <= nv < 64
    if (!kOutDirect && jl) {
#pragma unroll
      for (int k = 0; k < 3; k++) { vj[k] = xanchor[3 * tid + k]; vj[3 + k] = xaxis[3 * tid + k]; }
    }
    if (!kOutDirect2 && sl) {
#pragma unroll
      for (int k = 0; k < 3; k++) vs[k] = sxpos[3 * tid + k];
#pragma unroll
      for (int k = 0; k < 9; k++) vs[3 + k] = sxmat[9 * tid + k];
    }
    if (dl) {
      vd[0] = qfrc_bias[tid]; vd[1] = qfrc_passive[tid]; vd[2] = qfrc_act[tid]; vd[3] = qfrc_smooth[tid];
      vd[4] = qfrc_con[tid]; vd[5] = qacc_smooth[tid]; vd[6] = qacc[tid];
    }
    if (!kOutDirect && jl) {
      const long long o = (long long)W * nj + tid;
#pragma unroll
      for (int k = 0; k < 3; k++) { DP(xanchor)[3 * o + k] = vj[k]; DP(xaxis)[3 * o + k] = vj[3 + k]; }
    }
    // sites: compact (nworld, nsite), or inside a wider per-world array after
    // site_off static sites (mjh_data.site_wstride; the host wrote those once)
    float* const o_sxpos = d.site_wstride ? d.site_xpos : DP(site_xpos);
    float* const o_sxmat = d.site_wstride ? d.site_xmat : DP(site_xmat);
    const long long s_row = d.site_wstride ? (long long)W * d.site_wstride + d.site_off : (long long)W * Z.nsite;
    for (int st = tid; sl && !kOutDirect2; st += NT) {  // sites beyond the first 64: one more round each
      const long long o = s_row + st;
#pragma unroll
      for (int k = 0; k < 3; k++) o_sxpos[3 * o + k] = vs[k];
#pragma unroll
      for (int k = 0; k < 9; k++) o_sxmat[9 * o + k] = vs[3 + k];
      if (st + NT >= Z.nsite) break;
#pragma unroll
      for (int k = 0; k < 3; k++) vs[k] = sxpos[3 * (st + NT) + k];
#pragma unroll
      for (int k = 0; k < 9; k++) vs[3 + k] = sxmat[9 * (st + NT) + k];
    }
    if (dl) {
      const long long o = (long long)W * nv + tid;
      DP(qfrc_bias)[o] = vd[0]; DP(qfrc_passive)[o] = vd[1]; DP(qfrc_actuator)[o] = vd[2]; DP(qfrc_smooth)[o] = vd[3];
      DP(qfrc_constraint)[o] = vd[4]; DP(qacc_smooth)[o] = vd[5]; DP(qacc)[o] = vd[6]; DP(qacc_warmstart)[o] = vd[6];
    }
  }
  for (int ci = tid; !kOutDirect2 && ci < ncon; ci += NT) {
    float c[22];
    int ic[4];
    c[0] = con_dist[ci];
#pragma unroll
    for (int k = 0; k < 3; k++) c[1 + k] = con_pos[3 * ci + k];
#pragma unroll
    for (int k = 0; k < 9; k++) c[4 + k] = con_frame[9 * ci + k];
#pragma unroll
    for (int k = 0; k < 5; k++) c[13 + k] = con_fric[5 * ci + k];
    c[18] = con_imargin[ci];
    ic[0] = con_dim[ci]; ic[1] = con_geom[2 * ci]; ic[2] = con_geom[2 * ci + 1]; ic[3] = con_efcadr[ci];
    const long long o = W * Z.nconmax + ci;
    DP(contact_dist)[o] = c[0];
#pragma unroll
    for (int k = 0; k < 3; k++) DP(contact_pos)[3 * o + k] = c[1 + k];
#pragma unroll
    for (int k = 0; k < 9; k++) DP(contact_frame)[9 * o + k] = c[4 + k];
#pragma unroll
    for (int k = 0; k < 5; k++) DP(contact_friction)[5 * o + k] = c[13 + k];
    DP(contact_includemargin)[o] = c[18];
    DP(contact_dim)[o] = ic[0];
    DP(contact_geom)[2 * o] = ic[1];
    DP(contact_geom)[2 * o + 1] = ic[2];
    DP(contact_efc_address)[o] = ic[3];
  }
  for (int r = tid; r < nefc; r += NT) {
    const int ty = efc_type[r], id = efc_id[r];
    const float ps = efc_pos[r], dd = efc_D[r], ar = efc_aref[r], fo = efc_force[r];
    const long long o = W * Z.njmax + r;
    DP(efc_type)[o] = ty;
    DP(efc_id)[o] = id;
    DP(efc_pos)[o] = ps;
    DP(efc_D)[o] = dd;
    DP(efc_aref)[o] = ar;
    DP(efc_force)[o] = fo;
  }
  if (tid == 0) {
    DP(ncon)[W] = ncon;
    DP(nefc)[W] = nefc;
    DP(solver_niter)[W] = niter;
    DP(solver_lstrace)[3 * W] = (int)lstr0;
    DP(solver_lstrace)[3 * W + 1] = (int)lstr1;
    DP(solver_lstrace)[3 * W + 2] = (int)lstr2;
  }

  // ---------------------------------------------------------------- integration
  PROF(8);
  if (STEP) {
    const float dt = m.timestep;
    float* qa_int = tmp;
    if (m.integrator == MJH_INT_IMPLICITFAST) {
      mass_rows_to<NVP, PKL>(Mm, Lm, nv, ldm);
      for (int i = tid; i < nv; i += NT) Lm[lofs<PKL>(i, ldm) + i] += dt * dof_damping[i];
      wsync();
      for (int i = tid; i < nu; i += NT) {
        if (IMG_I(actuator_forcelimited)[i]) {
          const float f = act_force[i];
          if (f <= IMG_F(actuator_forcerange)[2 * i] || f >= IMG_F(actuator_forcerange)[2 * i + 1]) continue;
        }
        const int dof = IMG_I(jnt_dofadr)[IMG_I(actuator_trnid)[i]];
        const float g = IMG_F(actuator_gear)[i];
        atomicAdd(&Lm[lofs<PKL>(dof, ldm) + dof], -dt * g * g * IMG_F(actuator_biasprm)[10 * i + 2]);
      }
      for (int i = tid; i < nv; i += NT) qa_int[i] = qfrc_smooth[i] + qfrc_con[i];
      ldl_factor_reg<NVP, PKL>(Lm, nv, ldm);
      ldl_solve_reg<NVP, PKL>(Lm, nv, ldm, qa_int);
    } else {
      float anyd = 0.f;
      for (int i = tid; i < nv; i += NT) anyd += dof_damping[i] > 0.f ? 1.f : 0.f;
      anyd = bsum<NT>(anyd, red);
      if (anyd > 0.f) {
        mass_rows_to<NVP, PKL>(Mm, Lm, nv, ldm);
        for (int i = tid; i < nv; i += NT) Lm[lofs<PKL>(i, ldm) + i] += dt * dof_damping[i];
        symv_u<NT, NVP>(Mm, nv, ldm, qacc, qa_int);
        ldl_factor_reg<NVP, PKL>(Lm, nv, ldm);
        ldl_solve_reg<NVP, PKL>(Lm, nv, ldm, qa_int);
      } else {
        for (int i = tid; i < nv; i += NT) qa_int[i] = qacc[i];
        wsync();
      }
    }
    for (int i = tid; i < nv; i += NT) qvel[i] += dt * qa_int[i];
    wsync();
    for (int j = tid; j < nj; j += NT) {
      const int q0 = IMG_I(jnt_qposadr)[j], v0 = IMG_I(jnt_dofadr)[j];
      if (IMG_I(jnt_type)[j] == 0) {
        qpos[q0] += dt * qvel[v0];
        qpos[q0 + 1] += dt * qvel[v0 + 1];
        qpos[q0 + 2] += dt * qvel[v0 + 2];
        float q[4] = {qpos[q0 + 3], qpos[q0 + 4], qpos[q0 + 5], qpos[q0 + 6]};
        float om[3] = {qvel[v0 + 3], qvel[v0 + 4], qvel[v0 + 5]};
        const float ang = dt * normalize3(om);
        float qr[4];
        axis_angle(qr, om, ang);
        quat_normalize(q);
        quat_mul(q, q, qr);
        quat_normalize(q);
        qpos[q0 + 3] = q[0]; qpos[q0 + 4] = q[1]; qpos[q0 + 5] = q[2]; qpos[q0 + 6] = q[3];
      } else if (IMG_I(jnt_type)[j] == 1) {  // ball: mju_quatIntegrate
        float q[4] = {qpos[q0], qpos[q0 + 1], qpos[q0 + 2], qpos[q0 + 3]};
        float om[3] = {qvel[v0], qvel[v0 + 1], qvel[v0 + 2]};
        const float ang = dt * normalize3(om);
        float qr[4];
        axis_angle(qr, om, ang);
        quat_normalize(q);
        quat_mul(q, q, qr);
        quat_normalize(q);
        qpos[q0] = q[0]; qpos[q0 + 1] = q[1]; qpos[q0 + 2] = q[2]; qpos[q0 + 3] = q[3];
      } else {
        qpos[q0] += dt * qvel[v0];
      }
    }
    wsync();
    for (int i = tid; i < nq; i += NT) DP(qpos)[W * nq + i] = qpos[i];
    for (int i = tid; i < nv; i += NT) DP(qvel)[W * nv + i] = qvel[i];
    const float now = DP(time)[W] + dt;  // every lane: the value lane 0 stores
    if (tid == 0) DP(time)[W] = now;
    // fused contact-sensor timers (mjh_data.at_*; ContactSensor.
    // _update_air_time_tracking, contact_sensor.py:327-367): lane j, slot j
    if (d.at_cur_air != nullptr && tid < d.at_k) {
      const long long t = (long long)W * d.at_k + tid;
      const float el = now - d.at_last_time[W];
      const bool is_c = DP(sensordata)[W * Z.nsensordata + d.at_cols[tid]] > 0.f;
      const float ca = d.at_cur_air[t], cc = d.at_cur_con[t];
      if (ca > 0.f && is_c) d.at_last_air[t] = ca + el;
      d.at_cur_air[t] = is_c ? 0.f : ca + el;
      if (cc > 0.f && !is_c) d.at_last_con[t] = cc + el;
      d.at_cur_con[t] = is_c ? cc + el : 0.f;
    }
    if (d.at_cur_air != nullptr) {
      wsync();
      if (tid == 0) d.at_last_time[W] = now;
    }
  }

  // non-finite check on the new state
  PROF(9);
  {
    float bad = 0.f;
    for (int i = tid; i < nq; i += NT) bad += isfinite(qpos[i]) ? 0.f : 1.f;
    for (int i = tid; i < nv; i += NT) bad += (isfinite(qvel[i]) && isfinite(qacc[i])) ? 0.f : 1.f;
    bad = bsum<NT>(bad, red);
    if (tid == 0) {
      const int f = ints[I_FLAGS] | (bad > 0.f ? MJH_FLAG_NONFINITE : 0);
      DP(flags)[W] = f;
      DP(flags_acc)[W] |= f;  // sticky until the caller clears it (overflow/NaN statistics)
    }
  }
  }  // velocity / solver stage
  };  // tail
  if constexpr (kTwoTier) {
    if (big)
      tail(std::integral_constant<bool, true>{});
    else
      tail(std::integral_constant<bool, false>{});
  } else {
    (void)big;
    tail(std::integral_constant<bool, false>{});
  }
  if constexpr (!PERSIST) return;
  }  // world loop
}

#undef DP
__global__ void repeat_kernel(float* dst, const float* src, long long nelem, long long total) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
    dst[i] = src[i % nelem];
}

// ---- model image packing ------------------------------------------------------
// One workgroup per model field copies it into the packed image (all fields in
// parallel, ~µs); launched ahead of every step so in-place edits of shared
// model fields take effect at the next step, as with MuJoCo Warp.
// World visiting order for the step launch that follows (mjh_order_worlds'
// rule: descending (niter + 2) * nefc of the previous step in 256 buckets of
// 16), run by one extra workgroup of the pack launch.
constexpr int kPackOrderBuckets = 256;
__device__ void order_worlds_block(const int* __restrict__ niter, const int* __restrict__ nefc, long long* __restrict__ order,
                                   long long n) {
  __shared__ int cnt[kPackOrderBuckets];
  __shared__ int base[kPackOrderBuckets];
  for (int b = threadIdx.x; b < kPackOrderBuckets; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    const int key = (niter[e] + 2) * nefc[e];
    atomicAdd(&cnt[kPackOrderBuckets - 1 - min(key >> 4, kPackOrderBuckets - 1)], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < kPackOrderBuckets; b++) {
      base[b] = acc;
      acc += cnt[b];
    }
  }
  __syncthreads();
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    const int key = (niter[e] + 2) * nefc[e];
    order[atomicAdd(&base[kPackOrderBuckets - 1 - min(key >> 4, kPackOrderBuckets - 1)], 1)] = e;
  }
}

__global__ __launch_bounds__(1024) void pack_kernel(const mjh_model m, const ImgOff io, const int* niter, const int* nefc_w,
                                                   long long* order, long long nworld) {
  if ((int)blockIdx.x == io.nfields) {  // extra workgroup 1: the collision pairs' records
    if (MJH_PAIR_REC) {
      int* rec = reinterpret_cast<int*>(m.image) + io.pair_rec;
      for (int p = threadIdx.x; p < m.npair; p += blockDim.x) {
        const int g1 = m.pair_geom1[p], g2 = m.pair_geom2[p];
        const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
        const float mg = fmaxf(m.geom_margin[g1], m.geom_margin[g2]);
        // the same float operations, in the same order, as the test it replaces
        const float reach = t1 == 0 ? mg + m.geom_rbound[g2] : mg + m.geom_rbound[g1] + m.geom_rbound[g2];
        int* r = rec + 8 * p;
        r[0] = g1; r[1] = g2; r[2] = m.geom_colslot[g1]; r[3] = m.geom_colslot[g2];
        r[4] = t1; r[5] = t2; r[6] = __float_as_int(mg); r[7] = __float_as_int(reach);
      }
    }
    return;
  }
  if ((int)blockIdx.x == io.nfields + 1) {  // extra workgroup 2: world order
    order_worlds_block(niter, nefc_w, order, nworld);
    return;
  }
#define X_SZ(name) const int name = m.name;
  MJH_MODEL_SIZES(X_SZ)
#undef X_SZ
  (void)nchain; (void)ncolgeom; (void)npair; (void)nsensor; (void)nmocap; (void)nconmax; (void)njmax; (void)na;
  (void)nsensordata; (void)nq; (void)nv; (void)nu; (void)nbody; (void)njnt; (void)ngeom; (void)nsite;
  unsigned int* img = reinterpret_cast<unsigned int*>(m.image);
  if (blockIdx.x == 0 && threadIdx.x == 0) img[io.img_words] = 0u;  // the step launch's world-claim counter
  int f = 0;
#define X_PACK(type, name, count)                                                          \
  if ((int)blockIdx.x == f) {                                                              \
    const int words = (int)((count) * (int)(sizeof(type) / 4));                            \
    const unsigned int* src = reinterpret_cast<const unsigned int*>(m.name);               \
    for (int i = threadIdx.x; i < words; i += blockDim.x) img[io.name + i] = src[i];       \
    return;                                                                                \
  }                                                                                        \
  f++;
  MJH_MODEL_ARRAYS(X_PACK)
  MJH_MODEL_WARRAYS(X_PACK)
#undef X_PACK
}

// Debug copies of the last step/forward's mass matrix and constraint Jacobian
// out of each world's global scratch (where the step keeps them): qM (nv x nv)
// and efc_J (njmax x nv, rows < nefc). One workgroup per world.
__global__ __launch_bounds__(256) void debug_fields_kernel(const float* scratch, long long scratch_words, const int* nefc,
                                                          int nv, int ldm, int ldj, int offM, int offJ, int njmax,
                                                          float* qM, float* efc_J) {
  const long long w = blockIdx.x;
  const float* G = scratch + w * scratch_words;
  for (int i = threadIdx.x; i < nv * nv; i += blockDim.x) qM[w * nv * nv + i] = G[offM + (i / nv) * ldm + i % nv];
  const int ne = min(nefc[w], njmax);
  for (int i = threadIdx.x; i < ne * nv; i += blockDim.x)
    efc_J[w * (long long)njmax * nv + i] = G[offJ + (i / nv) * ldj + i % nv];
}

// ---- host side ---------------------------------------------------------------
inline int nvp_of(int nv) { return nv <= 20 ? 20 : (nv <= 36 ? 36 : 64); }
ImgOff make_imgoff(const mjh_model* m) {
  ImgOff io;
  std::memset(&io, 0, sizeof(io));
#define X_SZ(name) const int name = m->name;
  MJH_MODEL_SIZES(X_SZ)
#undef X_SZ
  (void)nchain; (void)ncolgeom; (void)npair; (void)nsensor; (void)nmocap; (void)nconmax; (void)njmax; (void)na;
  (void)nsensordata; (void)nq; (void)nv; (void)nu; (void)nbody; (void)njnt; (void)ngeom; (void)nsite;
  int off = 0, nf = 0;
#define X_OFF(type, name, count)                            \
  io.name = off;                                            \
  off += (((count) * (int)(sizeof(type) / 4)) + 1) & ~1;    \
  nf++;
  MJH_MODEL_ARRAYS(X_OFF)
  MJH_MODEL_WARRAYS(X_OFF)
#undef X_OFF
  // per collision pair, 8 words written by the pack launch from the geom arrays:
  // [geom1, geom2, colslot1, colslot2 | type1, type2, margin, reach] (reach: the
  // bounding-sphere test's right-hand side), two 16-byte loads per lane in the
  // collision pass instead of three dependent rounds of loads
  io.pair_rec = (off + 3) & ~3;
  off = io.pair_rec + (MJH_PAIR_REC ? 8 * m->npair : 0);
  io.img_words = (off + 3) & ~3;
  io.nfields = nf;
#define X_W(type, name, count) io.w_##name = -1;
  MJH_MODEL_WARRAYS(X_W)
#undef X_W
  return io;
}

// Per-world layout: arrays go to LDS (`off`) or to the global scratch
// (`goff`) according to the region table Rg. `budget` = LDS words available to
// one world; the constraint-row capacity is what fits (LDS rows) or njmax.
Layout make_layout(const mjh_model* m, int budget, int wpb) {
  Layout L;
  std::memset(&L, 0, sizeof(L));
  int off = 0, goff = 0;
  auto al = [](int n) { return (n + 3) & ~3; };  // 16-byte alignment (float4 rows, int64 masks)
#define TAKE(name, n)                 \
  do {                                \
    if (Rg::name) {                   \
      L.name = goff; goff += al(n);   \
    } else {                          \
      L.name = off; off += al(n);     \
    }                                 \
  } while (0)
  const int nv = m->nv, nb = m->nbody, nj = m->njnt;
  // rows 16-byte aligned with an odd float4 count: ds_read_b128 on a row per lane
  // lands on distinct bank quads (conflict-free), and row reads vectorise
  int ld = nvp_of(nv);  // == kernel's NVP (rows loaded whole into registers)
  if (((ld >> 2) & 1) == 0) ld += 4;
  L.ldm = ld;
  L.ldj = ld;
  TAKE(qpos, m->nq);
  // dof vectors padded to NVP: the unrolled row dots read them whole
  const int nvv = nvp_of(nv);
  TAKE(qvel, nvv); TAKE(qacc, nvv); TAKE(qacc_smooth, nvv); TAKE(qfrc_smooth, nvv);
  TAKE(qfrc_bias, nvv); TAKE(qfrc_con, nvv); TAKE(qfrc_passive, nvv); TAKE(qfrc_act, nvv);
  TAKE(grad, nvv); TAKE(search, nvv); TAKE(Ma, nvv); TAKE(Mv, nvv); TAKE(tmp, nvv); TAKE(tmp2, nvv);
  TAKE(xpos, 3 * nb); TAKE(xquat, 4 * nb); TAKE(xmat, 9 * nb); TAKE(xipos, 3 * nb);
  TAKE(ximat, 9 * nb); TAKE(subtree_com, 3 * nb); TAKE(cinert, 10 * nb); TAKE(crb, 10 * nb);
  TAKE(cvel, 6 * nb); TAKE(cacc, 6 * nb); TAKE(cfrc, 6 * nb);
  TAKE(xanchor, 3 * nj); TAKE(xaxis, 3 * nj); TAKE(cdof, 6 * nv); TAKE(cdof_dot, 6 * nv);
  TAKE(cgpos, 3 * m->ncolgeom); TAKE(cgmat, 9 * m->ncolgeom);
  TAKE(sxpos, 3 * m->nsite); TAKE(sxmat, 9 * m->nsite);
  const int lwords = pack_l(wpb) ? lrow(nvp_of(nv)) : nv * L.ldm;
  TAKE(M, nv * L.ldm); TAKE(L, lwords);
  TAKE(act_force, m->nu);
  const int C = m->nconmax;
  L.ncap = C;
  TAKE(con_pos, 3 * C); TAKE(con_frame, 9 * C); TAKE(con_dist, C); TAKE(con_fric, 5 * C);
  TAKE(con_solref, 2 * C); TAKE(con_solimp, 5 * C); TAKE(con_imargin, C); TAKE(con_dim, C);
  TAKE(con_geom, 2 * C); TAKE(con_efcadr, C);
  L.red = off; off += al(16);
  L.ints = off; off += al(8);
  // constraint rows: as many as fit in the remaining LDS budget (rows in LDS)
  // or njmax (rows in global scratch)
  // LDS words per constraint row (16-byte alignment padding is absorbed by
  // the 32-word slack below)
  const int per_row_lds = (Rg::J ? 0 : L.ldj) + !Rg::efc_D + !Rg::efc_R + !Rg::efc_aref + !Rg::efc_jaref +
                          !Rg::efc_jv + !Rg::efc_force + !Rg::efc_fl + !Rg::efc_pos + !Rg::efc_type + !Rg::efc_id +
                          2 * !Rg::efc_mask + !Rg::efc_h + !Rg::arow + !Rg::ash;
  int rcap = m->njmax, lcap = rcap;
  if (per_row_lds > 0) {
    const int r = (budget - off - 64) / per_row_lds;
    if (r < lcap) lcap = r;
  }
  if (cu_worlds(wpb) && g_lds_row_cap > 0 && g_lds_row_cap < lcap) lcap = g_lds_row_cap;
  if (lcap < 1) lcap = 1;
  // 8-world workgroups: rows beyond the LDS are dropped (flagged as overflow);
  // one-world and whole-CU workgroups: up to njmax, beyond lcap in global scratch (BIG)
  if (!cu_worlds(wpb)) rcap = lcap;
  L.rcap = rcap;
  L.lcap = lcap;
  // LDS-resident row arrays take lcap rows, global ones rcap
#define TAKER(name, extra) TAKE(name, (Rg::name ? rcap : lcap) + (extra))
  // elliptic cones: the cone Hessian's virtual rows after row rcap (at most one per row)
  TAKE(J, (m->cone == 1 ? 2 * rcap : rcap) * L.ldj);
  TAKER(efc_D, 0); TAKER(efc_R, 0); TAKER(efc_aref, 0); TAKER(efc_jaref, 0);
  TAKER(efc_jv, 0); TAKER(efc_force, 0); TAKER(efc_fl, 0); TAKE(efc_pos, rcap);
  TAKER(efc_type, 0); TAKE(efc_id, rcap);
  TAKE(efc_mask, 2 * rcap);
  TAKER(efc_h, 0); TAKER(arow, 4); TAKER(ash, 4);
#undef TAKER
  TAKE(sidx, 64);
  TAKE(cg_g, nvv); TAKE(cg_mg, nvv);
#undef TAKE
  L.total = al(off);
  // split-step handoff (global scratch): the factor of M, the rows' position
  // parameters, counters and the reuse snapshot
  auto gt = [&](int n) { const int o = goff; goff += al(n); return o; };
  // the BIG worlds' row arrays (one-world workgroups with lcap < rcap)
  {
    const bool two = cu_worlds(wpb);  // allocated whatever lcap is: the scratch size does not depend on it
    L.g_efc_D = two ? gt(rcap) : 0; L.g_efc_R = two ? gt(rcap) : 0; L.g_efc_aref = two ? gt(rcap) : 0;
    L.g_efc_jaref = two ? gt(rcap) : 0; L.g_efc_jv = two ? gt(rcap) : 0; L.g_efc_force = two ? gt(rcap) : 0;
    L.g_efc_fl = two ? gt(rcap) : 0; L.g_efc_type = two ? gt(rcap) : 0; L.g_efc_h = two ? gt(rcap) : 0;
    L.g_arow = two ? gt(rcap + 4) : 0; L.g_ash = two ? gt(rcap + 4) : 0;
  }
  L.h_L = gt(lwords);
  L.h_type = gt(rcap); L.h_fl = gt(rcap); L.h_D = gt(rcap); L.h_R = gt(rcap);
  L.h_aref = gt(rcap); L.h_b = gt(rcap); L.h_jv = gt(rcap);
  L.h_ints = gt(8);
  // PGS only (the dual's matrices; a model solved by Newton or CG allocates nothing)
  L.pgs_ar = m->solver == kSolverPGS ? gt(rcap * rcap) : 0;
  L.pgs_mj = m->solver == kSolverPGS ? gt(rcap * L.ldj) : 0;
  L.h_snap = gt(7 + m->nq + 7 * m->nmocap);
  // the position kernel's LDS per world: qpos, reductions, counters
  L.pred = al(m->nq);
  L.pints = L.pred + al(16);
  L.ptotal = L.pints + al(8);
  L.gtotal = al(goff) + 64;  // +256 B keeps worlds' spans on separate cache lines
  return L;
}

constexpr int kLdsBytes = 160 * 1024;
constexpr int kPosWorldsPerBlock = MJH_PWPB;

struct Plan {
  ImgOff io;
  Layout lo;
  size_t shmem;
  size_t shmem_pos;  // the split position kernel's
};

Plan make_plan(const mjh_model* m) {
  Plan p;
  const int wpb = wpb_of_nvp(nvp_of(m->nv));
  p.io = make_imgoff(m);
  const int img_lds = img_global(wpb) ? 0 : p.io.img_words;
  // MJH_WPCU / wpb workgroups share a CU's LDS (one-world workgroups: MJH_WPCU
  // per CU, the waves per SIMD the launch bound's VGPR budget allows); 8-world
  // workgroups: one per CU
  const int budget = (kLdsBytes / 4 / (wpb < 8 ? MJH_WPCU / wpb : 1) - img_lds) / wpb;
  p.lo = make_layout(m, budget, wpb);
  p.shmem = (size_t)(img_lds + wpb * p.lo.total) * 4;
  p.shmem_pos = (size_t)((img_global(kPosWorldsPerBlock) ? 0 : p.io.img_words) + kPosWorldsPerBlock * p.lo.ptotal) * 4;
  return p;
}

void plan_to_ints(const Plan& p, const mjh_model* m, int* v) {
  v[0] = nvp_of(m->nv);
  int k = 1;
#define X_SZP(name) v[k++] = m->name;
  MJH_MODEL_SIZES(X_SZP)
#undef X_SZP
  std::memcpy(v + k, &p.lo, sizeof(Layout));
  std::memcpy(v + k + kLayoutInts, &p.io, sizeof(ImgOff));
}

// whether every data array sits in one slab at nworld * data_offsets() (the
// Simulation's allocation), so a specialised instance may derive the pointers
bool data_is_slab(const mjh_model* m, const mjh_data* d) {
  Sizes z;
#define X_SZH(name) z.name = m->name;
  MJH_MODEL_SIZES(X_SZH)
#undef X_SZH
  const DataOff o = data_offsets(z);
  const char* base = reinterpret_cast<const char*>(d->qpos);
  bool ok = true;
  // site outputs in a wider array (site_wstride) are addressed through their pointers
  const bool wide = d->site_wstride != 0;
#define X_SL(type, name, count)                                                                  \
  ok = ok && ((wide && (std::strcmp(#name, "site_xpos") == 0 || std::strcmp(#name, "site_xmat") == 0)) || \
              reinterpret_cast<const char*>(d->name) == base + 4ll * o.name * d->nworld);
  MJH_DATA_ARRAYS(X_SL)
#undef X_SL
  return ok;
}

// the specialised instance whose plan equals this model's, or -1
int find_spec(const Plan& p, const mjh_model* m) {
  if (MJH_NSPEC == 0) return -1;
  if (m->cone == 1) return -1;  // elliptic cones: generic instances only
  if (m->solver == kSolverPGS) return -1;  // PGS: generic instances only
  int v[kPlanInts];
  plan_to_ints(p, m, v);
  for (int k = 0; k < MJH_NSPEC; k++)
    if (std::memcmp(v, kSpecPlan[k], sizeof(v)) == 0) return k;
  return -1;
}

// FNV-1a over the model and data descriptors: any change of an option scalar,
// size or buffer address invalidates every world's position snapshot
unsigned long long launch_key(const mjh_model* m, const mjh_data* d) {
  unsigned long long h = 1469598103934665603ull;
  auto eat = [&h](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  };
  eat(m, sizeof(*m));
  eat(d, offsetof(mjh_data, at_last_time));  // the fused sensor timers do not affect the position stage
  // the site-output layout does (the position stage writes the sites there)
  eat(&d->site_wstride, sizeof(d->site_wstride));
  eat(&d->site_off, sizeof(d->site_off));
  return h;
}

// Launch plugins (mjh_register_spec_plugin): model-specialised instances built
// for a plan after the library was (mjlab_amd/sim/jit.py compiles this file with
// -DMJH_PLUGIN and a one-plan table when a Simulation's model matches no entry of
// mjh_spec_table.h, and registers the library's mjh_plugin_step here). A plugin
// is taken on the same conditions as a built-in specialisation: exact plan
// match, slab data layout, pyramidal cones, Newton or CG.
typedef int (*PluginFn)(int step, const int* plan, const mjh_model* m, const mjh_data* d, const unsigned char* gate,
                        void* stream, int reuse, unsigned long long key);
struct PluginEntry {
  int plan[kPlanInts];
  PluginFn fn;
};
std::vector<PluginEntry> g_plugins;

int find_plugin(const Plan& p, const mjh_model* m) {
  if (g_plugins.empty() || MJH_SPLIT != 0 || m->cone == 1 || m->solver == kSolverPGS) return -1;
  int v[kPlanInts];
  plan_to_ints(p, m, v);
  for (size_t k = 0; k < g_plugins.size(); k++)
    if (std::memcmp(v, g_plugins[k].plan, sizeof(v)) == 0) return (int)k;
  return -1;
}

// one step/forward launch of MODE (0 fused, 1 position, 2 velocity/solver)
template <int WPB, bool STEP, int NVP, int SPEC, bool SLAB, int MODE>
void launch_mode(const Plan& p, const mjh_model* m, const mjh_data* d, const unsigned char* gate, hipStream_t s,
                 int reuse, unsigned long long key) {
  auto kern = step_kernel<WPB, NVP, SPEC, SLAB, MODE>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    attr = true;
  }
  int blocks = (d->nworld + WPB - 1) / WPB;
  if (MJH_PERSIST && MODE == 0) {
    // persistent: as many workgroups as are resident at once
    static int resident = 0;
    if (resident == 0) {
      int per_cu = 0, dev = 0, ncu = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), 64 * WPB, p.shmem);
      resident = (per_cu > 0 ? per_cu : 1) * (ncu > 0 ? ncu : 1);
    }
    if (blocks > resident) blocks = resident;
  }
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * WPB), MODE == 1 ? p.shmem_pos : p.shmem, s, *m, *d, p.lo, p.io, gate,
                     reuse, key, STEP ? 1 : 0);
}

template <bool STEP, int NVP, int SPEC, bool SLAB>
void launch_step(const Plan& p, const mjh_model* m, const mjh_data* d, const unsigned char* gate, hipStream_t s) {
  if constexpr (MJH_SPLIT != 0) {
    launch_mode<kPosWorldsPerBlock, STEP, NVP, SPEC, SLAB, 1>(p, m, d, gate, s, g_pos_reuse ? 1 : 0, launch_key(m, d));
    launch_mode<wpb_of_nvp(NVP), STEP, NVP, SPEC, SLAB, 2>(p, m, d, gate, s, 0, 0ull);
  } else {
    launch_mode<wpb_of_nvp(NVP), STEP, NVP, SPEC, SLAB, 0>(p, m, d, gate, s, g_pos_reuse ? 1 : 0, launch_key(m, d));
  }
}

template <bool STEP, int K>
void launch_spec(int k, const Plan& p, const mjh_model* m, const mjh_data* d, const unsigned char* gate, hipStream_t s) {
  if constexpr (K < MJH_NSPEC) {
    if (k != K) return launch_spec<STEP, K + 1>(k, p, m, d, gate, s);
    launch_step<STEP, kSpecNvp[K], K, true>(p, m, d, gate, s);
  }
}

template <bool STEP>
int launch(const mjh_model* m, const mjh_data* d, const unsigned char* gate, void* stream) {
  if (mjh_model_check(m) != 0) return 1;
  if (d->nworld <= 0) return 0;
  Plan p = make_plan(m);
  if (!d->scratch || d->scratch_words < p.lo.gtotal) {
    g_err = "data scratch buffer missing or too small (mjh_scratch_words)";
    return 1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nvp = nvp_of(m->nv);
  const bool order = g_auto_order && d->world_order != nullptr && d->nworld > 1;
  // 1024 threads: the order workgroup's counting sort is the launch's long pole
  if (!g_keep_image)
    hipLaunchKernelGGL(pack_kernel, dim3(p.io.nfields + 1 + (order ? 1 : 0)), dim3(1024), 0, s, *m, p.io, d->solver_niter,
                       d->nefc, const_cast<long long*>(d->world_order), (long long)d->nworld);
  // specialised instances assume the slab data layout (data_is_slab)
  const bool slab = !g_disable_spec && data_is_slab(m, d);
  const int k = slab ? find_spec(p, m) : -1;
  const int kp = (slab && k < 0) ? find_plugin(p, m) : -1;
  if (k >= 0) {
    launch_spec<STEP, 0>(k, p, m, d, gate, s);
  } else if (kp >= 0) {
    const int r = g_plugins[kp].fn(STEP ? 1 : 0, g_plugins[kp].plan, m, d, gate, stream, g_pos_reuse ? 1 : 0,
                                   launch_key(m, d));
    if (r != 0) {
      g_err = "specialised plugin launch failed (code " + std::to_string(r) + ")";
      return 2;
    }
  } else if (nvp == 20)
    launch_step<STEP, 20, -1, false>(p, m, d, gate, s);
  else if (nvp == 36)
    launch_step<STEP, 36, -1, false>(p, m, d, gate, s);
  else
    launch_step<STEP, 64, -1, false>(p, m, d, gate, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("step launch failed: ") + hipGetErrorString(e);
    return 2;
  }
  return 0;
}

}  // namespace

#ifdef MJH_PLUGIN
// ---- plugin build (-DMJH_PLUGIN, MJH_SPEC_TABLE = a one-plan table) ------------
// Exports only the launch of its specialised instance; the main library
// packs the model image and orders the worlds before calling it.
extern "C" {
int mjh_plugin_abi(void) { return MJH_ABI_VERSION; }

int mjh_plugin_plan(int* out, int cap) {
  if (MJH_NSPEC != 1 || cap < kPlanInts) return -1;
  for (int i = 0; i < kPlanInts; i++) out[i] = kSpecPlan[0][i];
  return kPlanInts;
}

int mjh_plugin_step(int step, const int* plan, const mjh_model* m, const mjh_data* d, const unsigned char* gate,
                    void* stream, int reuse, unsigned long long key) {
  if constexpr (MJH_NSPEC == 1) {
    // the plan the caller matched (its own build state, e.g. a test's LDS row
    // cap, entered it) must be this plugin's; the launch geometry follows from it
    if (!plan || std::memcmp(plan, kSpecPlan[0], sizeof(int) * kPlanInts) != 0 || !data_is_slab(m, d)) return 3;
    Plan p;
    std::memcpy(&p.lo, plan + 1 + kSizeInts, sizeof(Layout));
    std::memcpy(&p.io, plan + 1 + kSizeInts + kLayoutInts, sizeof(ImgOff));
    constexpr int WPB = wpb_of_nvp(kSpecNvp[0]);
    p.shmem = (size_t)((img_global(WPB) ? 0 : p.io.img_words) + WPB * p.lo.total) * 4;
    p.shmem_pos = (size_t)((img_global(kPosWorldsPerBlock) ? 0 : p.io.img_words) + kPosWorldsPerBlock * p.lo.ptotal) * 4;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    constexpr int NVP = kSpecNvp[0];
    if (step)
      launch_mode<wpb_of_nvp(NVP), true, NVP, 0, true, 0>(p, m, d, gate, s, reuse, key);
    else
      launch_mode<wpb_of_nvp(NVP), false, NVP, 0, true, 0>(p, m, d, gate, s, reuse, key);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  return 4;
}
}  // extern "C"
#else
extern "C" {

int mjh_abi_version(void) { return MJH_ABI_VERSION; }

int mjh_register_spec_plugin(void* fn, const int* plan, int nplan) {
  if (!fn || !plan || nplan != kPlanInts) {
    g_err = "mjh_register_spec_plugin: null function or plan of the wrong length";
    return -1;
  }
  for (size_t k = 0; k < g_plugins.size(); k++)
    if (std::memcmp(plan, g_plugins[k].plan, sizeof(int) * kPlanInts) == 0) {
      g_plugins[k].fn = reinterpret_cast<PluginFn>(fn);
      return (int)k;
    }
  PluginEntry e;
  std::memcpy(e.plan, plan, sizeof(e.plan));
  e.fn = reinterpret_cast<PluginFn>(fn);
  g_plugins.push_back(e);
  return (int)g_plugins.size() - 1;
}

int mjh_plugin_index(const mjh_model* m) {
  if (!m) return -1;
  return find_spec(make_plan(m), m) >= 0 ? -1 : find_plugin(make_plan(m), m);
}

const char* mjh_last_error(void) { return g_err.c_str(); }

size_t mjh_sizeof_model(void) { return sizeof(mjh_model); }
size_t mjh_sizeof_data(void) { return sizeof(mjh_data); }

// + 4 words after the image: the step launch's world-claim counter (+ padding)
int mjh_image_words(const mjh_model* m) { return make_imgoff(m).img_words + 4; }

int mjh_model_check(const mjh_model* m) {
  if (!m) { g_err = "null model"; return 1; }
  if (m->nv > 63 || m->nbody > 63) { g_err = "device path supports nv <= 63 and nbody <= 63"; return 1; }
  if (m->nconmax <= 0 || m->njmax <= 0) { g_err = "nconmax and njmax must be positive"; return 1; }
  Plan p = make_plan(m);
  if (!m->image || m->image_words < p.io.img_words + 4) { g_err = "model image buffer missing or too small (mjh_image_words)"; return 1; }
  if (p.shmem > (size_t)kLdsBytes) { g_err = "model image + per-world scratch exceed LDS"; return 1; }
  if (p.lo.rcap < 8) { g_err = "too little LDS left for constraint rows"; return 1; }
  // elliptic rows need the constraint Jacobian in global scratch (a preset that
  // keeps J in LDS builds pyramidal rows only)
  if (m->cone == 1 && !Rg::J) { g_err = "elliptic cones need a build with J in global scratch (MJH_PRESET)"; return 1; }
  if (m->solver == kSolverPGS && m->cone == 1) { g_err = "the PGS solver supports pyramidal cones only"; return 1; }
  if (m->solver == kSolverPGS && (!Rg::J || !Rg::M)) { g_err = "the PGS solver needs a build with J and M in global scratch"; return 1; }
  g_err.clear();
  return 0;
}

int mjh_scratch_bytes(const mjh_model* m) { return (int)make_plan(m).shmem; }

int mjh_efc_capacity(const mjh_model* m) { return make_plan(m).lo.rcap; }
int mjh_lds_rows(const mjh_model* m) { return make_plan(m).lo.lcap; }

extern const int mjh_layout_ints = kLayoutInts;  // for tools/gen_spec.py

int mjh_set_specialization(int enable) {
  g_disable_spec = enable == 0;
  return 0;
}

int mjh_set_world_ordering(int on) {
  g_auto_order = on != 0;
  return 0;
}

int mjh_set_position_reuse(int on) {
  // a preset that keeps position-stage arrays in LDS cannot reuse them
  g_pos_reuse = on != 0 && kPositionStageGlobal;
  return MJH_SPLIT ? 1 : 0;
}

int mjh_split_step(void) { return MJH_SPLIT; }

int mjh_set_lds_row_cap(int rows) {
  g_lds_row_cap = rows > 0 ? rows : 0;
  return 0;
}

int mjh_spec_index(const mjh_model* m) { return find_spec(make_plan(m), m); }

int mjh_data_is_slab(const mjh_model* m, const mjh_data* d) { return data_is_slab(m, d) ? 1 : 0; }

int mjh_plan_ints(const mjh_model* m, int* out, int cap) {
  const Plan p = make_plan(m);
  int v[kPlanInts];
  plan_to_ints(p, m, v);
  if (cap < kPlanInts) return -1;
  for (int i = 0; i < kPlanInts; i++) out[i] = v[i];
  return kPlanInts;
}

long long mjh_scratch_words(const mjh_model* m) { return make_plan(m).lo.gtotal; }

#ifdef MJH_PROFILE
// diagnostics (profile builds only; not part of the ABI): the parallel line
// search's candidate costs at iteration MJH_LSDBG_IT, (nworld, 32) floats
extern "C" int mjh_set_lsdbg_buffer(void* ptr) {
  float* p = reinterpret_cast<float*>(ptr);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_lsdbg), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
#endif

int mjh_set_profile_buffer(void* ptr) {
#ifdef MJH_PROFILE
  unsigned long long* p = reinterpret_cast<unsigned long long*>(ptr);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), &p, sizeof(p)) == hipSuccess ? 0 : 1;
#else
  (void)ptr;
  return 1;
#endif
}

int mjh_step(const mjh_model* m, const mjh_data* d, void* stream) { return launch<true>(m, d, nullptr, stream); }

int mjh_forward(const mjh_model* m, const mjh_data* d, void* stream) { return launch<false>(m, d, nullptr, stream); }

int mjh_step_keep_image(const mjh_model* m, const mjh_data* d, void* stream) {
  // a persistent build (MJH_PERSIST) resets its world-claim counter in the pack
  // launch, so it always packs (the image is rebuilt: same results, one launch more)
  g_keep_image = MJH_PERSIST == 0;
  const int r = launch<true>(m, d, nullptr, stream);
  g_keep_image = false;
  return r;
}

int mjh_forward_gated(const mjh_model* m, const mjh_data* d, const unsigned char* gate, void* stream) {
  if (!gate) { g_err = "null gate"; return 1; }
  return launch<false>(m, d, gate, stream);
}

int mjh_debug_fields(const mjh_model* m, const mjh_data* d, float* qM, float* efc_J, void* stream) {
  if (mjh_model_check(m) != 0) return 1;
  if (!Rg::M || !Rg::J) { g_err = "this build keeps M or J in LDS (MJH_PRESET): no debug copy"; return 1; }
  if (!qM || !efc_J || !d->scratch) { g_err = "null output or scratch"; return 1; }
  if (d->nworld <= 0) return 0;
  const Plan p = make_plan(m);
  hipLaunchKernelGGL(debug_fields_kernel, dim3(d->nworld), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), d->scratch,
                     d->scratch_words, d->nefc, m->nv, p.lo.ldm, p.lo.ldj, p.lo.M, p.lo.J, m->njmax, qM, efc_J);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { g_err = hipGetErrorString(e); return 2; }
  return 0;
}

int mjh_repeat(float* dst, const float* src, long long nelem, int nworld, void* stream) {
  if (nelem <= 0 || nworld <= 0) return 0;
  long long total = nelem * (long long)nworld;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(repeat_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), dst, src, nelem, total);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { g_err = hipGetErrorString(e); return 2; }
  return 0;
}

}  // extern "C"
#endif  // MJH_PLUGIN
