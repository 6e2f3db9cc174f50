// ecnf_kernels.hpp — the device side of libecnf_hip.so: the ODE integrator and vector-field kernels and their
// templated launchers (included by ecnf_hip.hip, which either instantiates every compiled shape itself or, in
// the split build, declares them extern; and by ecnf_part.hip, one translation unit per compiled shape).
//
//   vf_kernel        one EGNN evaluation (+ JVPs) per molecule      <- cnf.apply / jax.vjp
//   integrate_kernel the whole ODE solve, one launch: each workgroup integrates its MPW molecules end to end
//                    (Euler / Dopri5 fixed step / Dopri5 + PID per molecule), state in LDS, the EGNN eval
//                    as a device function                            <- diffrax.diffeqsolve
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ecnf.h"
#include "egnn_eval.hpp"

namespace ecnf {

// ---------------------------------------------------------------------------------------------------
// Dopri5 tableau (diffrax 2023: Shampine's embedded pair, FSAL)
// ---------------------------------------------------------------------------------------------------
__constant__ float kA[6][6] = {
    {(float)(1.0 / 5), 0, 0, 0, 0, 0},
    {(float)(3.0 / 40), (float)(9.0 / 40), 0, 0, 0, 0},
    {(float)(44.0 / 45), (float)(-56.0 / 15), (float)(32.0 / 9), 0, 0, 0},
    {(float)(19372.0 / 6561), (float)(-25360.0 / 2187), (float)(64448.0 / 6561), (float)(-212.0 / 729), 0, 0},
    {(float)(9017.0 / 3168), (float)(-355.0 / 33), (float)(46732.0 / 5247), (float)(49.0 / 176),
     (float)(-5103.0 / 18656), 0},
    {(float)(35.0 / 384), 0.0f, (float)(500.0 / 1113), (float)(125.0 / 192), (float)(-2187.0 / 6784),
     (float)(11.0 / 84)}};
__constant__ float kC[7] = {0.0f, (float)(1.0 / 5), (float)(3.0 / 10), (float)(4.0 / 5), (float)(8.0 / 9), 1.0f, 1.0f};
__constant__ float kBerr[7] = {(float)(35.0 / 384 - 1951.0 / 21600),
                               0.0f,
                               (float)(500.0 / 1113 - 22642.0 / 50085),
                               (float)(125.0 / 192 - 451.0 / 720),
                               (float)(-2187.0 / 6784 + 12231.0 / 42400),
                               (float)(11.0 / 84 - 649.0 / 6300),
                               (float)(-1.0 / 60.0)};

struct SolveP {
  int solver, div, adaptive, max_steps;
  float tau0, tau1, dirf, dt0, rtol, atol, dtmin;
  // exact trace: block 1 runs the edges at the tangent's atom as dual tiles and every edge as a primal tile
  // (egnn_eval sparse_a; set by the host where it pays: the M <= 128 split tangent kernels, >= 3 tiles per molecule
  // per dual tile)
  int sparse1;
  // exact trace with sparse1: per-molecule cache of the primal edge aggregates of blocks 1 and K ([molecule slot of
  // the grid][N M + 2 N D] floats), written by the first JVP pass of an evaluation and read by the other ND - D - 1
  // (the primal is the same in every pass), which then run only the dual tiles of those blocks.  nullptr: off.
  // pcache_slots: molecule slots the buffer holds (>= grid x MPW; device-checked build: ECNF_DCHECK bit 6)
  float* pcache;
  int pcache_slots;
  // team (latency) mode of the primal kernels (egnn_eval.hpp team_exchange): team.G > 1 workgroups per molecule,
  // MPW = 1, grid = batch x G (a cooperative launch: every member co-resident)
  TeamP team;
  // re-dealt adaptive solves (ecnf_hip.hip integrate_impl): `order` maps launch slots to batch molecules (nullptr:
  // the identity) and *nslots (device memory) is the number of occupied slots (nullptr: B); `state` [B][state_stride]
  // holds a molecule's solver state at a step boundary (SolverState), stored when the launch stops after
  // `chunk_steps` > 0 step controls (or ends) and loaded instead of the initial state when `resume` is set
  const int* order;
  const int* nslots;
  float* state;
  int state_stride, chunk_steps, resume;
};

// one molecule's solver state at a step boundary (stage 1 of the next step, FSAL k1 in kx[0]): y [ND], k1 [ND], then
// these scalars (ints as their bits)
enum SolverState { kSsLp = 0, kSsKl, kSsTau, kSsDt, kSsTnext, kSsAtmin, kSsNfe, kSsSteps, kSsStatus, kSsActive, kSsCount };
__host__ __device__ inline int solver_state_stride(int ND) { return align4(2 * ND + kSsCount); }
// batch molecule of launch slot slot0 + m (re-dealt solves: through the slot order)
__device__ __forceinline__ int mol_index(const int* order, int slot0, int m) {
  return order ? order[slot0 + m] : slot0 + m;
}
// kernels that can stop and resume (every integrate kernel but the strict-fp32 M = 256 tangent one, whose 92 spilled
// registers crash the compiler's AGPR-copy rewrite pass once the state copies are added; its solves run in one launch)
__host__ __device__ constexpr bool chunkable(int NF, int NT, int P) { return !(P == 1 && NF == 8 && NT == 1); }

// solver state in LDS, after the eval region
struct SolverLds {
  float *ys, *vout, *tin, *tout, *y, *eps, *kx;   // [MPW][ND] each, kx [7][MPW][ND]
  float *ts, *divv, *lp, *kl, *tau, *tnext, *dt, *h, *l1, *h0;   // [MPW] (kl: [7][MPW])
  int *active, *atmin, *nfe, *steps, *status, *keep, *any;
  // the phase machine's uniform control state (integrate_kernel): [0] Euler tau, [1] Euler next tau (float bits),
  // [2] Euler steps, [3] phase, [4] stage.  Read from LDS on both sides of every evaluation instead of being held in
  // registers across it (held, they spilled)
  int* ctl;
};

__host__ __device__ inline int solver_lds_floats(int MPW, int ND) {
  return 13 * align4(MPW * ND) + 16 * align4(MPW) + 8 * align4(MPW) + 4 + 8;
}

__device__ inline SolverLds carve_solver(float* p, int MPW, int ND) {
  SolverLds st;
  const int a = align4(MPW * ND), b = align4(MPW);
  st.ys = p; p += a;  st.vout = p; p += a;  st.tin = p; p += a;  st.tout = p; p += a;
  st.y = p; p += a;   st.eps = p; p += a;   st.kx = p; p += 7 * a;
  st.ts = p; p += b;  st.divv = p; p += b;  st.lp = p; p += b;   st.kl = p; p += 7 * b;
  st.tau = p; p += b; st.tnext = p; p += b; st.dt = p; p += b;   st.h = p; p += b;
  st.l1 = p; p += b;  st.h0 = p; p += b;
  int* q = reinterpret_cast<int*>(p);
  st.active = q; q += b; st.atmin = q; q += b; st.nfe = q; q += b; st.steps = q; q += b;
  st.status = q; q += b; st.keep = q; q += b; st.any = q; q += 4;
  st.ctl = q;
  return st;
}

__device__ __forceinline__ float uniform_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, x)));
}

// (solver_sizes(): egnn_eval.hpp)
__device__ __forceinline__ int solver_size(int k) { return __builtin_amdgcn_readfirstlane(solver_sizes()[k]); }

// tau1 passes an empty asm (wave-uniform) so the threshold tau1 - 1e-6 is formed at each use: hoisted out of the solver
// loop it was a loop-invariant VGPR that spilled in the 256-register kernels
__device__ inline float clip_end(float tn, float tau1) {
  int tb = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, tau1));
  asm volatile("" : "+s"(tb));
  const float t1 = __builtin_bit_cast(float, tb);
  return tn > t1 - 1e-6f ? t1 : tn;
}

// embedding ids of one molecule (LDS [N]) in [0, n_features)?  Out-of-range ids are replaced by 0 (memory safety).
__device__ inline bool check_features(const Net& net, int* f) {
  bool ok = true;
  for (int i = 0; i < net.N; ++i)
    if (f[i] < 0 || f[i] >= net.nfeat) {
      ok = false;
      f[i] = 0;
    }
  return ok;
}

// one evaluation of the joint field g(tau, y) = dir * f(dir * tau, y) at (st.ts, st.ys) for every molecule
// of the workgroup; writes kx_out [MPW][ND] and kl_out [MPW].  Exactly one egnn_eval call site (it is inlined).
template <int NF, int NT, int L, int D, int P, bool TEAM, bool COLS, bool BN>
__device__ __forceinline__ void joint_field(const Net& net, const Lds& s, const SolverLds& st, const SolveP& sp,
                                            float* kx_out, float* kl_out, const TeamCtx* tm, int* tepoch) {
  constexpr int kThreads = kernel_threads<NF, NT, P, COLS>();
  // per-thread indices are re-derived (opaque_tid) on each side of the evaluation: kept live across it, they spill
  const int MPW = solver_size(0), ND = solver_size(1);
  int tid = opaque_tid();
  // NT == 0: one primal eval; Hutchinson: one JVP along eps; exact: the trace of J from ND - D JVPs along e_k,
  // k >= D.  The field only sees relative positions and subtracts the input mean (egnn.py:176-188), so
  // v(x + s 1) = v(x) - s exactly, i.e. J T_c = -T_c for the translations T_c = sum_a e_(a,c).  In the basis
  // {T_c} u {e_k, k >= D} the dual vectors are e_(0,c) and e_k - e_(k mod D), hence
  //   tr J = sum_{k >= D} (J_kk - J_(k mod D),k) - D
  // with J_(k mod D),k the atom-0 component of the same JVP column (D fewer evaluations than the ND unit JVPs).
  // (sp.div re-read through an empty asm at each use: the hoisted flag and -D were loop-invariant VGPRs that spilled)
  const bool exact = NT && opaque_u(sp.div) != ECNF_DIV_HUTCHINSON;
  const int nrep = exact ? ND - D : 1;
  if (tid < MPW) st.divv[tid] = exact ? -(float)D : 0.f;
  for (int k0 = 0; k0 < nrep; ++k0) {
    const int k = exact ? k0 + D : k0;
    tid = opaque_tid();
    if constexpr (NT) {
      if (sp.div == ECNF_DIV_HUTCHINSON) {
        for (int i = tid; i < MPW * ND; i += kThreads) st.tin[i] = st.eps[i];
      } else {
        for (int i = tid, NDo = opaque_u(ND); i < MPW * NDo; i += kThreads) st.tin[i] = ((i % NDo) == k) ? 1.0f : 0.0f;
      }
      __syncthreads();
    }
    // exact: the unit tangent e_k sits on atom k / D, so block 1 (whose node features carry no tangent) has nonzero
    // edge tangents only on the 2(N - 1) edges at that atom
    const bool sparse = exact && sp.sparse1;
    float* pc = sparse && sp.pcache
                    ? sp.pcache + (size_t)blockIdx.x * MPW * (net.N * (NF * 32) + 2 * net.N * D)
                    : nullptr;
    ECNF_DCHECK(!pc || (int)(blockIdx.x + 1) * MPW <= sp.pcache_slots, 6);
    egnn_eval<NF, NT, L, D, P, TEAM, COLS, BN>(net, s, st.ys, st.ts, st.tin, st.vout, st.tout, st.active, sparse ? k / D : -1,
                                     pc, k0 == 0 ? 1 : 2, tm, tepoch);
    tid = opaque_tid();
    if constexpr (NT) {
      if (tid < MPW) {
        if (sp.div == ECNF_DIV_HUTCHINSON) {
          float acc = 0.f;
          for (int c = 0; c < ND; ++c) acc += st.tout[tid * ND + c] * st.eps[tid * ND + c];
          st.divv[tid] = acc;
        } else {
          st.divv[tid] += st.tout[tid * ND + k] - st.tout[tid * ND + k % D];
        }
      }
    }
  }
  tid = opaque_tid();
  for (int i = tid; i < MPW * ND; i += kThreads) kx_out[i] = sp.dirf * st.vout[i];
  if (tid < MPW) {
    kl_out[tid] = sp.dirf * st.divv[tid];
    if (st.active[tid]) st.nfe[tid] += 1;
  }
  __syncthreads();
}

// diffrax rms_norm over the leaves of one molecule's state: (x, logp) when the divergence is tracked
// (get_log_prob / sample_and_log_prob_cnf), x alone for sample_cnf (sample_and_log_prob.py:28-37 has y0 = x0)
__device__ inline float rms_state(float sumsq_x, float l, int ND, bool track) {
  return track ? sqrtf((sumsq_x + l * l) / (float)(ND + 1)) : sqrtf(sumsq_x / (float)ND);
}

enum Phase { kEuler = 0, kInit0 = 1, kInit1 = 2, kFsal = 3, kStage = 4 };

// The whole solve as a phase machine around ONE field evaluation per loop trip.  TEAM: the team (latency) mode
// instantiation (egnn_eval.hpp team_exchange; launched only with sp.team.G > 1, compiled for team_shape)
template <int NF, int NT, int L, int D, int P, bool TEAM = false, bool COLS = false, bool BN = false>
__global__ __launch_bounds__((kernel_threads<NF, NT, P, COLS>())) __attribute__((amdgpu_waves_per_eu(Geo<NF, NT, P>::WPE))) void integrate_kernel(Net net, SolveP sp, const float* __restrict__ y0,
                                                                  const int32_t* __restrict__ feat,
                                                                  const float* __restrict__ eps, float* y1,
                                                                  float* dlogp, int32_t* nfe_out,
                                                                  int32_t* status_out, int B) {
  constexpr int kThreads = kernel_threads<NF, NT, P, COLS>();
  extern __shared__ float smem[];
  const int tid = (int)threadIdx.x, MPW = net.MPW, ND = net.ND, N = net.N;
  const Lds s = carve_lds<NT, Geo<NF, NT, P, BN>::kSplitN, Geo<NF, NT, P, BN>::kNoP>(net, smem);
  const SolverLds st = carve_solver(s.tail, MPW, ND);
  // team mode (MPW = 1; only member 0 writes outputs): the K G workgroups [0, K G) are the members of slots [0, K),
  // in groups of 8 teams whose members sit 8 (or the last group's team count) blocks apart -- member r of team 8 q + j
  // is block 8 G q + nl r + j, nl = min(8, K - 8 q) -- so that under the round-robin block -> XCD dispatch a team's
  // members share one XCD and its L2 (the exchange's write-through stores and loads then stay in that L2;
  // MI355X_MICROARCH.md: placement is for speed only, the hand-off protocol does not depend on it).  K = B, or
  // *sp.team.nteam for the re-dealt solve's tail teams, whose other slots run alone from block K G on (G = 1, no
  // exchange)
  TeamCtx team_ctx;
  constexpr bool team = TEAM;
  team_ctx.p = sp.team;
  team_ctx.T = 0;
  team_ctx.r = 0;
  team_ctx.G = 1;
  if constexpr (team) {
    const int G = sp.team.G, b = (int)blockIdx.x;
    const int K = sp.team.nteam ? *sp.team.nteam : B;
    if (b < K * G) {
      const int q = b / (8 * G), nl = min(8, K - 8 * q), rem = b - 8 * G * q;
      team_ctx.r = rem / nl;
      team_ctx.T = 8 * q + (rem - team_ctx.r * nl);
      team_ctx.G = G;
    } else {
      team_ctx.T = K + (b - K * G);
    }
  }
  const TeamCtx* tm = team ? &team_ctx : nullptr;
  if constexpr (team) {
    if (threadIdx.x == 0) *team_stop_flag() = 0;   // (stop-and-team: no verdict before the first exchange)
  }
  int tepoch = 0;
  const bool writer_wg = team_ctx.r == 0;
  // launch slots slot0 .. slot0 + nmol - 1; slot j integrates batch molecule sp.order[j] (re-dealt solves) or j
  const int slot0 = team ? team_ctx.T : (int)blockIdx.x * MPW;
  const int nmol = min(MPW, (sp.nslots ? *sp.nslots : B) - slot0);
  if (nmol <= 0) return;   // a re-dealt launch keeps the batch's grid; slots past the unfinished molecules are empty
  ECNF_DCHECK((int)(s.tail - smem) + solver_lds_floats(MPW, ND) <= net.lds_floats, 0);
  ECNF_DCHECK(nmol >= 1 && nmol <= MPW, 5);

  // zero the eval scratch and the solver state (aggregates must start at +0; padding rows and the solver slots of
  // padding molecules stay finite: a resumed launch loads kx[0] / kl of the occupied slots only)
  for (int i = tid; i < (int)(s.tail - smem) + solver_lds_floats(MPW, ND); i += kThreads) smem[i] = 0.f;
  __syncthreads();
  for (int i = tid; i < MPW * ND; i += kThreads) {
    const int m = i / ND;
    const size_t g = m < nmol ? (size_t)mol_index(sp.order, slot0, m) * ND + (i - m * ND) : 0;
    st.y[i] = m < nmol ? y0[g] : 0.f;
    st.eps[i] = (m < nmol && eps) ? eps[g] : 0.f;
  }
  for (int i = tid; i < MPW * N; i += kThreads) {
    const int m = i / N;
    s.feat[i] = m < nmol ? feat[(size_t)mol_index(sp.order, slot0, m) * N + (i - m * N)] : 0;
  }
  if (tid < MPW) {
    st.lp[tid] = 0.f;
    st.tau[tid] = sp.tau0;
    st.active[tid] = tid < nmol ? 1 : 0;
    st.atmin[tid] = 0;
    st.nfe[tid] = 0;
    st.steps[tid] = 0;
    st.status[tid] = ECNF_OK;
    st.dt[tid] = sp.dt0;
    st.tnext[tid] = clip_end(fminf(sp.tau0 + sp.dt0, sp.tau1), sp.tau1);
  }
  if (tid == 0) {
    solver_sizes()[0] = MPW;
    solver_sizes()[1] = ND;
    solver_sizes()[2] = (int)(s.tail - smem);
    // Euler: ConstantStepSize, all molecules share the (uniform) time grid
    st.ctl[0] = __builtin_bit_cast(int, sp.tau0);
    st.ctl[1] = __builtin_bit_cast(int, clip_end(sp.tau0 + sp.dt0, sp.tau1));
    st.ctl[2] = 0;
    st.ctl[3] = sp.solver == ECNF_SOLVER_EULER ? kEuler : (sp.adaptive ? kInit0 : kFsal);
    st.ctl[4] = 1;
    st.ctl[5] = 0;   // step controls in this launch (chunked solves)
    if (chunkable(NF, NT, P) && sp.resume) {   // a resumed molecule continues at stage 1 of its next step
      st.ctl[3] = kStage;
      st.ctl[4] = 1;
    }
  }
  if (chunkable(NF, NT, P) && sp.resume) {
    for (int i = tid; i < nmol * ND; i += kThreads) {
      const int m = i / ND, c = i - m * ND;
      const float* S = sp.state + (size_t)mol_index(sp.order, slot0, m) * sp.state_stride;
      st.y[i] = S[c];
      st.kx[i] = S[ND + c];
    }
    if (tid < nmol) {
      const float* S = sp.state + (size_t)mol_index(sp.order, slot0, tid) * sp.state_stride + 2 * ND;
      st.lp[tid] = S[kSsLp];
      st.kl[tid] = S[kSsKl];
      st.tau[tid] = S[kSsTau];
      st.dt[tid] = S[kSsDt];
      st.tnext[tid] = S[kSsTnext];
      st.atmin[tid] = __builtin_bit_cast(int, S[kSsAtmin]);
      st.nfe[tid] = __builtin_bit_cast(int, S[kSsNfe]);
      st.steps[tid] = __builtin_bit_cast(int, S[kSsSteps]);
      st.status[tid] = __builtin_bit_cast(int, S[kSsStatus]);
      st.active[tid] = __builtin_bit_cast(int, S[kSsActive]);
    }
  }
  __syncthreads();
  // device-side input check (no host sync on the call path): a molecule with an embedding id outside
  // [0, n_features) reports ECNF_E_INVALID (nn.Embed would index out of range) and is solved with id 0
  if (tid < nmol && !check_features(net, s.feat + tid * N)) st.status[tid] = ECNF_E_INVALID;
  __syncthreads();


#ifdef ECNF_STAMPS
  if (tid == 0) {
    for (int i = 0; i < 32; ++i) s.stamps[i] = 0;
    s.stamps[31] = __builtin_amdgcn_s_memtime();
    s.stamps[30] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  while (true) {
    const int tid = opaque_tid();   // shadows the kernel-level tid: nothing per-thread stays live across an eval
    const int MPW = solver_size(0), ND = solver_size(1);   // (likewise the sizes, the solver-state pointers)
    const SolverLds st = carve_solver(smem + solver_size(2), MPW, ND);
    const int a = align4(MPW * ND), b = align4(MPW);
    // the control state, wave-uniform (SGPRs)
    float e_tau = uniform_f(__builtin_bit_cast(float, st.ctl[0])), e_tn = uniform_f(__builtin_bit_cast(float, st.ctl[1]));
    int e_steps = __builtin_amdgcn_readfirstlane(st.ctl[2]);
    int phase = __builtin_amdgcn_readfirstlane(st.ctl[3]), stage = __builtin_amdgcn_readfirstlane(st.ctl[4]);
    STAMP(s, kStSolver);
    // ------------------------------------------------ inputs of this evaluation
    float* kx_out;
    float* kl_out;
    if (phase == kEuler) {
      if (!(e_tau < sp.tau1)) break;
      if (++e_steps > sp.max_steps) {
        if (tid < nmol) st.status[tid] = ECNF_E_MAX_STEPS;
        break;
      }
      for (int i = tid; i < MPW * ND; i += kThreads) st.ys[i] = st.y[i];
      if (tid < MPW) st.ts[tid] = sp.dirf * e_tau;
      kx_out = st.kx; kl_out = st.kl;
    } else if (phase == kInit0 || phase == kFsal) {
      for (int i = tid; i < MPW * ND; i += kThreads) st.ys[i] = st.y[i];
      if (tid < MPW) st.ts[tid] = sp.dirf * st.tau[tid];
      kx_out = st.kx; kl_out = st.kl;
    } else if (phase == kInit1) {
      for (int i = tid; i < MPW * ND; i += kThreads) st.ys[i] = st.y[i] + st.h0[i / ND] * st.kx[i];
      if (tid < MPW) st.ts[tid] = sp.dirf * (st.tau[tid] + st.h0[tid]);
      kx_out = st.kx + a; kl_out = st.kl + b;
    } else {
      if (stage == 1) {
        if (tid == 0) {
          int any = 0;
          for (int m = 0; m < MPW; ++m) any |= st.active[m];
          if constexpr (TEAM) {
            // stop-and-team: stop at this step boundary once few molecules are left (a team: member 0's verdict from
            // the last exchange, the same for every member)
            if (sp.team.fin) {
              const bool stop = team_ctx.G > 1 ? *team_stop_flag() != 0
                                               : *sp.team.nsl - __hip_atomic_load((ECNF_GLOBAL int*)sp.team.fin,
                                                                                  __ATOMIC_RELAXED,
                                                                                  __HIP_MEMORY_SCOPE_AGENT) <=
                                                     sp.team.stop_left;
              if (stop) any |= 2;
            }
          }
          *st.any = any;
        }
        if (tid < MPW) st.h[tid] = st.tnext[tid] - st.tau[tid];
        __syncthreads();
        if ((*st.any & 1) == 0 || (*st.any & 2)) break;
        // chunked solve: stop at this step boundary once the launch has done its step controls (state stored below)
        const int chunk = chunkable(NF, NT, P) ? opaque_u(sp.chunk_steps) : 0;
        if (chunk > 0 && __builtin_amdgcn_readfirstlane(st.ctl[5]) >= chunk) break;
      }
      for (int i = tid; i < MPW * ND; i += kThreads) {
        float acc = 0.f;
        for (int j = 0; j < stage; ++j) acc += kA[stage - 1][j] * st.kx[j * a + i];
        st.ys[i] = st.y[i] + st.h[i / ND] * acc;
      }
      if (tid < MPW) st.ts[tid] = sp.dirf * (st.tau[tid] + kC[stage] * st.h[tid]);
      kx_out = st.kx + stage * a; kl_out = st.kl + stage * b;
    }
    __syncthreads();

    joint_field<NF, NT, L, D, P, TEAM, COLS, BN>(net, s, st, sp, kx_out, kl_out, tm, &tepoch);

    // ------------------------------------------------ consume it
    {
    // per-thread indices, solver pointers and the control state re-derived after the evaluation (nothing of the
    // trip's first half stays live across it)
    const int tid = opaque_tid();
    const int MPW = solver_size(0), ND = solver_size(1);
    const SolverLds st = carve_solver(smem + solver_size(2), MPW, ND);
    const int a = align4(MPW * ND), b = align4(MPW);
    e_tau = uniform_f(__builtin_bit_cast(float, st.ctl[0]));
    e_tn = uniform_f(__builtin_bit_cast(float, st.ctl[1]));
    phase = __builtin_amdgcn_readfirstlane(st.ctl[3]);
    e_steps = __builtin_amdgcn_readfirstlane(st.ctl[2]) + (phase == kEuler ? 1 : 0);   // (this trip's Euler step)
    stage = __builtin_amdgcn_readfirstlane(st.ctl[4]);
    const float e_h = uniform_f(e_tn - e_tau);
    if (phase == kEuler) {
      for (int i = tid; i < MPW * ND; i += kThreads) st.y[i] = st.y[i] + e_h * st.kx[i];
      if (tid < MPW) st.lp[tid] = st.lp[tid] + e_h * st.kl[tid];
      e_tau = e_tn;
      e_tn = uniform_f(clip_end(e_tau + sp.dt0, sp.tau1));
    } else if (phase == kInit0) {
      // Hairer's initial step, part 1 (diffrax _select_initial_step)
      if (tid < MPW) {
        float sy = 0.f, sf = 0.f;
        for (int c = 0; c < ND; ++c) {
          const float yy = st.y[tid * ND + c];
          const float sc = sp.atol + fabsf(yy) * sp.rtol;
          sy += (yy / sc) * (yy / sc);
          sf += (st.kx[tid * ND + c] / sc) * (st.kx[tid * ND + c] / sc);
        }
        const float scl = sp.atol + fabsf(st.lp[tid]) * sp.rtol;
        const float d0 = rms_state(sy, st.lp[tid] / scl, ND, opaque_u(sp.div) != ECNF_DIV_NONE);
        const float d1 = rms_state(sf, st.kl[tid] / scl, ND, opaque_u(sp.div) != ECNF_DIV_NONE);
        const bool cond = (d0 < 1e-5f) || (d1 < 1e-5f);
        const float d1s = cond ? 1.0f : d1;
        st.h0[tid] = cond ? 1e-6f : 0.01f * (d0 / d1s);
        st.l1[tid] = d1;   // stash d1
      }
      phase = kInit1;
    } else if (phase == kInit1) {
      if (tid < MPW) {
        float s2 = 0.f;
        for (int c = 0; c < ND; ++c) {
          const float sc = sp.atol + fabsf(st.y[tid * ND + c]) * sp.rtol;
          const float df = (st.kx[a + tid * ND + c] - st.kx[tid * ND + c]) / sc;
          s2 += df * df;
        }
        const float scl = sp.atol + fabsf(st.lp[tid]) * sp.rtol;
        const float h0 = st.h0[tid];
        const float d1 = st.l1[tid];
        const float d2 = rms_state(s2, (st.kl[b + tid] - st.kl[tid]) / scl, ND, opaque_u(sp.div) != ECNF_DIV_NONE) / h0;
        const float maxd = fmaxf(d1, d2);
        const float h1 = maxd <= 1e-15f ? fmaxf(1e-6f, h0 * 1e-3f) : powf(0.01f / maxd, 0.2f);
        const float dt = fminf(100.0f * h0, h1);
        st.atmin[tid] = dt <= sp.dtmin ? 1 : 0;
        st.dt[tid] = fmaxf(dt, sp.dtmin);
        st.tnext[tid] = clip_end(fminf(st.tau[tid] + st.dt[tid], sp.tau1), sp.tau1);
      }
      phase = kFsal;
    } else if (phase == kFsal) {
      phase = kStage;
      stage = 1;
    } else if (stage < 6) {
      ++stage;
    } else {
      // st.ys holds y1 (the stage-7 input uses a_7 = b_sol): error estimate and step control per molecule
      if (tid < MPW) {
        const int m = tid;
        const float h = st.h[m];
        float accl = 0.f;
        for (int j = 0; j < 6; ++j) accl += kA[5][j] * st.kl[j * b + m];
        const float l1 = st.lp[m] + h * accl;
        st.l1[m] = l1;
        int keep = 1;
        float new_dt = sp.dt0;
        int new_atmin = 0;
        if (sp.adaptive) {
          float ssum = 0.f;
          for (int c = 0; c < ND; ++c) {
            float e = 0.f;
            for (int j = 0; j < 7; ++j) e += kBerr[j] * st.kx[j * a + m * ND + c];
            e = h * e;
            const float sc = sp.atol + fmaxf(fabsf(st.y[m * ND + c]), fabsf(st.ys[m * ND + c])) * sp.rtol;
            ssum += (e / sc) * (e / sc);
          }
          float el = 0.f;
          for (int j = 0; j < 7; ++j) el += kBerr[j] * st.kl[j * b + m];
          el = h * el;
          const float scl = sp.atol + fmaxf(fabsf(st.lp[m]), fabsf(l1)) * sp.rtol;
          const float err = rms_state(ssum, el / scl, ND, opaque_u(sp.div) != ECNF_DIV_NONE);
          keep = (err < 1.0f) || st.atmin[m];
          const float inv = 1.0f / err;
          float factor = 0.9f * powf(inv, 0.2f);
          factor = fminf(fmaxf(factor, keep ? 1.0f : 0.2f), 10.0f);
          if (isnan(factor)) factor = 1.0f;
          new_dt = h * factor;
          new_atmin = new_dt <= sp.dtmin ? 1 : 0;
          new_dt = fmaxf(new_dt, sp.dtmin);
        }
        st.keep[m] = keep && st.active[m];
        st.dt[m] = new_dt;
        st.h0[m] = (float)new_atmin;
      }
      __syncthreads();
      for (int i = tid; i < MPW * ND; i += kThreads) {
        const int m = i / ND;
        if (st.keep[m]) {
          st.y[i] = st.ys[i];
          st.kx[i] = st.kx[6 * a + i];
        }
      }
      if (tid < MPW) {
        const int m = tid;
        if (st.active[m]) {
          if (st.keep[m]) {
            st.lp[m] = st.l1[m];
            st.kl[m] = st.kl[6 * b + m];
            st.tau[m] = st.tnext[m];
          }
          st.atmin[m] = (int)st.h0[m];
          st.steps[m] += 1;
          st.tnext[m] = sp.adaptive ? clip_end(fminf(st.tau[m] + st.dt[m], sp.tau1), sp.tau1)
                                    : clip_end(st.tau[m] + sp.dt0, sp.tau1);
          if (!(st.tau[m] < sp.tau1)) {
            st.active[m] = 0;
          } else if (st.steps[m] >= sp.max_steps) {
            st.status[m] = ECNF_E_MAX_STEPS;
            st.active[m] = 0;
          }
          if constexpr (TEAM) {   // stop-and-team: one count per finished molecule (its member 0)
            if (sp.team.fin && !st.active[m] && team_ctx.r == 0)
              __hip_atomic_fetch_add((ECNF_GLOBAL int*)sp.team.fin, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      stage = 1;
      if (tid == 0) st.ctl[5] += 1;
    }
    if (tid == 0) {   // the control state of the next trip (read by every thread after the barrier)
      st.ctl[0] = __builtin_bit_cast(int, e_tau);
      st.ctl[1] = __builtin_bit_cast(int, e_tn);
      st.ctl[2] = e_steps;
      st.ctl[3] = phase;
      st.ctl[4] = stage;
    }
    __syncthreads();
    }   // consume
  }
  __syncthreads();
#ifdef ECNF_STAMPS
  if (threadIdx.x == 0) {
    STAMP(s, kStSolver);
    s.stamps[29] = __builtin_amdgcn_s_memrealtime() - s.stamps[30];
    for (int i = 0; i < kStCount; ++i) atomicAdd(&g_stamps[i], s.stamps[i]);
    atomicAdd(&g_stamps[29], s.stamps[29]);
    atomicAdd(&g_stamps[28], 1ull);
  }
#endif
  // failure detection: a final state that is not finite (activations beyond the fp16 range of the split GEMMs, an
  // overflowing field) is reported per molecule instead of passing as ECNF_OK.  (tid and the solver-state pointers
  // re-derived here: kept from the kernel's start, they would stay live across the whole solve and spill.)
  {
  const int tid = opaque_tid();
  const SolverLds st = carve_solver(smem + solver_size(2), MPW, ND);
  // chunked solve (or a stop-and-team launch): every molecule's state at this step boundary
  if (chunkable(NF, NT, P) && (sp.chunk_steps > 0 || (TEAM && sp.team.fin))) {
    for (int i = tid; i < nmol * ND; i += kThreads) {
      const int m = i / ND, c = i - m * ND;
      float* S = sp.state + (size_t)mol_index(sp.order, slot0, m) * sp.state_stride;
      S[c] = st.y[i];
      S[ND + c] = st.kx[i];
    }
    if (tid < nmol) {
      float* S = sp.state + (size_t)mol_index(sp.order, slot0, tid) * sp.state_stride + 2 * ND;
      S[kSsLp] = st.lp[tid];
      S[kSsKl] = st.kl[tid];
      S[kSsTau] = st.tau[tid];
      S[kSsDt] = st.dt[tid];
      S[kSsTnext] = st.tnext[tid];
      S[kSsAtmin] = __builtin_bit_cast(float, st.atmin[tid]);
      S[kSsNfe] = __builtin_bit_cast(float, st.nfe[tid]);
      S[kSsSteps] = __builtin_bit_cast(float, st.steps[tid]);
      S[kSsStatus] = __builtin_bit_cast(float, st.status[tid]);
      S[kSsActive] = __builtin_bit_cast(float, st.active[tid]);
    }
    __syncthreads();
  }
  if (tid < nmol && st.status[tid] == ECNF_OK) {
    bool fin = isfinite(st.lp[tid]);
    for (int c = 0; c < ND; ++c) fin = fin && isfinite(st.y[tid * ND + c]);
    if (!fin) st.status[tid] = ECNF_E_NONFINITE;
  }
  if constexpr (team) {
    // an exchange that timed out (a member not co-resident) leaves this molecule's results undefined
    if (tid == 0 && team_ctx.G > 1 &&
        __hip_atomic_load((ECNF_GLOBAL int*)(sp.team.timeout + team_ctx.T), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      st.status[0] = ECNF_E_HIP;
    __syncthreads();
    if (!writer_wg) return;
  }
  // (a molecule still unfinished at a chunk's end gets provisional outputs, overwritten by the launch that ends it)
  for (int i = tid; i < nmol * ND; i += kThreads) {
    const int m = i / ND;
    y1[(size_t)mol_index(sp.order, slot0, m) * ND + (i - m * ND)] = st.y[i];
  }
  if (tid < nmol) {
    const int bm = mol_index(sp.order, slot0, tid);
    if (dlogp) dlogp[bm] = st.lp[tid];
    if (nfe_out) nfe_out[bm] = st.nfe[tid];
    if (status_out) status_out[bm] = st.status[tid];
  }
  }
}

// one evaluation (and n_tangents JVPs) per molecule
template <int NF, int NT, int L, int D, int P, bool BN = false>
__global__ __launch_bounds__((Geo<NF, NT, P>::NTHR)) __attribute__((amdgpu_waves_per_eu(Geo<NF, NT, P>::WPE))) void vf_kernel(Net net, const float* __restrict__ x,
                                                           const float* __restrict__ t,
                                                           const int32_t* __restrict__ feat,
                                                           const float* __restrict__ tan_in, int ntan, float* v,
                                                           float* tan_out, int B) {
  constexpr int kThreads = Geo<NF, NT, P>::NTHR;
  extern __shared__ float smem[];
  const int tid = threadIdx.x, MPW = net.MPW, ND = net.ND, N = net.N;
  const Lds s = carve_lds<NT, Geo<NF, NT, P, BN>::kSplitN, Geo<NF, NT, P, BN>::kNoP>(net, smem);
  const SolverLds st = carve_solver(s.tail, MPW, ND);
  const int mol0 = blockIdx.x * MPW;
  const int nmol = min(MPW, B - mol0);
  ECNF_DCHECK((int)(s.tail - smem) + solver_lds_floats(MPW, ND) <= net.lds_floats, 0);
  ECNF_DCHECK(nmol >= 1 && nmol <= MPW, 5);
  for (int i = tid; i < (int)(s.tail - smem); i += kThreads) smem[i] = 0.f;
  __syncthreads();
  for (int i = tid; i < MPW * ND; i += kThreads) st.ys[i] = (i / ND) < nmol ? x[(size_t)mol0 * ND + i] : 0.f;
  for (int i = tid; i < MPW * N; i += kThreads) s.feat[i] = (i / N) < nmol ? feat[(size_t)mol0 * N + i] : 0;
  if (tid < MPW) st.ts[tid] = tid < nmol ? t[mol0 + tid] : 0.f;
  __syncthreads();
  // embedding ids outside [0, n_features): the molecule's outputs are NaN (no status output on this entry point)
  if (tid < MPW) st.keep[tid] = (tid < nmol && !check_features(net, s.feat + tid * N)) ? 1 : 0;
  __syncthreads();
  const float kNaN = __builtin_nanf("");
  if constexpr (NT == 0) {
    egnn_eval<NF, 0, L, D, P>(net, s, st.ys, st.ts, nullptr, st.vout, nullptr);
    for (int i = tid; i < nmol * ND; i += kThreads) v[(size_t)mol0 * ND + i] = st.keep[i / ND] ? kNaN : st.vout[i];
  } else {
    for (int k = 0; k < ntan; ++k) {
      for (int i = tid; i < MPW * ND; i += kThreads) {
        const int m = i / ND, c = i - m * ND;
        st.tin[i] = m < nmol ? tan_in[((size_t)(mol0 + m) * ntan + k) * ND + c] : 0.f;
      }
      __syncthreads();
      egnn_eval<NF, 1, L, D, P, false, false, BN>(net, s, st.ys, st.ts, st.tin, st.vout, st.tout);
      for (int i = tid; i < nmol * ND; i += kThreads) {
        const int m = i / ND, c = i - m * ND;
        tan_out[((size_t)(mol0 + m) * ntan + k) * ND + c] = st.keep[m] ? kNaN : st.tout[i];
        if (k == 0 && v) v[(size_t)mol0 * ND + i] = st.keep[m] ? kNaN : st.vout[i];
      }
      __syncthreads();
    }
  }
}

// shapes with a team-mode kernel (ecnf_hip.hip team_size): the split primal kernels of the BASELINE networks
// (QM9 M = 256, LJ13 M = 128, ALDP M = 64), and ALDP's split tangent kernel (Hutchinson solves: the re-dealt adaptive
// log_prob's tail teams, redeal_kernel; one molecule per workgroup)
constexpr bool team_shape(int M, int NT, int L, int D, int P) {
  return P == 0 && D == 3 &&
         (NT == 0 ? ((M == 256 && L == 4) || (M == 128 && L == 3) || (M == 64 && L == 2)) : (M == 64 && L == 2));
}

// shapes with a column-split team kernel (egnn_eval.hpp edge_tile_cols): the M = 256 team shape (QM9; 4 waves split
// its 8 output blocks)
constexpr bool cols_shape(int M, int NT, int L, int D, int P) { return team_shape(M, NT, L, D, P) && M == 256; }

// ---- templated launchers (one instantiation per compiled shape and tangent flag) ----
template <int NF, int NT, int L, int D, int P>
hipError_t launch_integrate(const Net& net, size_t lds, const SolveP& sp, const float* y0, const int32_t* feat,
                            const float* eps, float* y1, float* dlogp, int32_t* nfe, int32_t* status, int B,
                            hipStream_t stream) {
  if constexpr (team_shape(NF * 32, NT, L, D, P)) {
    if (sp.team.G > 1 && sp.team.nteam) {
      // the re-dealt solve's tail teams: slots [0, K) as teams of G, the rest alone (K <= nteam_max on the device).
      // Not cooperative: the grid exceeds the co-resident workgroups, but at most K (G - 1) < CUs members ever wait
      // for a partner, and every other workgroup runs to its end without waiting, so each partner is dispatched
      auto kt = integrate_kernel<NF, NT, L, D, P, true>;
      hipError_t e = hipFuncSetAttribute((const void*)kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(kt, dim3(B + sp.team.nteam_max * (sp.team.G - 1)), dim3(Geo<NF, NT, P>::NTHR), lds, stream,
                         net, sp, y0, feat, eps, y1, dlogp, nfe, status, B);
      return hipGetLastError();
    }
    if (sp.team.G > 1) {
    // team mode: the G members of a molecule wait on each other, so the launch must be co-resident; the cooperative
    // launch checks the grid against the occupancy query (hipErrorCooperativeLaunchTooLarge instead of a hang)
    auto kt = integrate_kernel<NF, NT, L, D, P, true>;
    if constexpr (cols_shape(NF * 32, NT, L, D, P)) {
      if (sp.team.cols) kt = integrate_kernel<NF, NT, L, D, P, true, true>;
    }
    if (sp.team.cols && !cols_shape(NF * 32, NT, L, D, P)) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute((const void*)kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    Net n = net;
    SolveP p = sp;
    const float* a_y0 = y0;
    const int32_t* a_feat = feat;
    const float* a_eps = eps;
    int a_B = B;
    void* args[] = {&n, &p, &a_y0, &a_feat, &a_eps, &y1, &dlogp, &nfe, &status, &a_B};
    const int nthr = sp.team.cols ? kernel_threads<NF, NT, P, true>() : Geo<NF, NT, P>::NTHR;
    return hipLaunchCooperativeKernel((const void*)kt, dim3(B * sp.team.G), dim3(nthr), args, lds, stream);
    }
  }
  if (sp.team.G > 1) return hipErrorInvalidValue;   // no team kernel for this shape (team_size never asks for one)
  auto k = integrate_kernel<NF, NT, L, D, P>;
  if constexpr (NT == 1 && NF == 4) {   // molecules of 34 .. 64 atoms: the wide (no P rows) form (Net::wide)
    if (net.wide) k = integrate_kernel<NF, NT, L, D, P, false, false, true>;
  }
  if (net.wide && !(NT == 1 && NF == 4)) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int grid = (B + net.MPW - 1) / net.MPW;
  hipLaunchKernelGGL(k, dim3(grid), dim3(Geo<NF, NT, P>::NTHR), lds, stream, net, sp, y0, feat, eps, y1, dlogp, nfe,
                     status, B);
  return hipGetLastError();
}

template <int NF, int NT, int L, int D, int P>
hipError_t launch_vf(const Net& net, size_t lds, const float* x, const float* t, const int32_t* feat,
                     const float* tan_in, int ntan, float* v, float* tan_out, int B, hipStream_t stream) {
  auto k = vf_kernel<NF, NT, L, D, P>;
  if constexpr (NT == 1 && NF == 4) {
    if (net.wide) k = vf_kernel<NF, NT, L, D, P, true>;
  }
  if (net.wide && !(NT == 1 && NF == 4)) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int grid = (B + net.MPW - 1) / net.MPW;
  hipLaunchKernelGGL(k, dim3(grid), dim3(Geo<NF, NT, P>::NTHR), lds, stream, net, x, t, feat, tan_in, ntan, v, tan_out,
                     B);
  return hipGetLastError();
}

// compiled shapes: (M, L, D) with tangent support where registers allow (M <= 128).  __graft_entry__.build()
// reads these two lists to compile one ecnf_part.hip translation unit per shape.
// ECNF_SHAPES: primal and tangent kernels in both GEMM arithmetics; ECNF_SHAPES_WIDE_TAN (M = 256): the same, the
// tangent kernels with per-edge phi_e.0 and sequential primal / tangent chain passes (Geo::kWideT split fp16,
// Geo::kWideT32 strict fp32)
#ifdef ECNF_DEV_LJ13_ONLY   // experiment builds (tools/build_variants.sh): the LJ13 shape only
#define ECNF_SHAPES(X) X(128, 3, 3)
#define ECNF_SHAPES_WIDE_TAN(X)
#elif defined(ECNF_DEV_M)       // experiment builds of one other shape (tools/build_timing.sh with DEVFLAGS)
#define ECNF_SHAPES(X) X(ECNF_DEV_M, ECNF_DEV_L, ECNF_DEV_D)
#define ECNF_SHAPES_WIDE_TAN(X)
#else
#define ECNF_SHAPES(X)  \
  X(128, 3, 3)          \
  X(128, 3, 2)          \
  X(128, 2, 3)          \
  X(128, 2, 2)          \
  X(64, 2, 3)           \
  X(64, 2, 2)           \
  X(64, 3, 3)           \
  X(64, 3, 2)

#define ECNF_SHAPES_WIDE_TAN(X) \
  X(256, 4, 3)                  \
  X(256, 3, 3)
#endif


// explicit instantiation (EXT = template) or instantiation declaration (EXT = extern template) of one shape
#define ECNF_INST_SHAPE(EXT, m, l, d, NTV, PV)                                                                \
  EXT hipError_t launch_integrate<m / 32, NTV, l, d, PV>(const Net&, size_t, const SolveP&, const float*,         \
                                                     const int32_t*, const float*, float*, float*, int32_t*, \
                                                     int32_t*, int, hipStream_t);                             \
  EXT hipError_t launch_vf<m / 32, NTV, l, d, PV>(const Net&, size_t, const float*, const float*, const int32_t*, \
                                              const float*, int, float*, float*, int, hipStream_t);

}  // namespace ecnf
