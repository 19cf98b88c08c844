// cf2sim_internal.h -- kernel parameter block and SoA field map shared by the HIP kernels
// and the C-ABI layer (not part of the public ABI; see include/cf2sim.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cf2sim_pack.h"

namespace cf2 {

// ---- float state fields: state_f[field * N + env] (DESIGN.md "State layout") ----
enum : int {
    F_POS = 0,          // 3  base position, world
    F_QUAT = 3,         // 4  base orientation (x,y,z,w), world
    F_VEL = 7,          // 3  base linear velocity, world
    F_OMEGA = 10,       // 3  bullet: angular velocity, world  | simple: body rates (drone.rpy_dot)
    F_RPY = 13,         // 3  simple only: integrated rpy (drone.rpy)
    F_MOTOR = 16,       // 4  first-order motor state x
    F_OU = 20,          // 4  OU thrust-noise state
    F_ABUF = 24,        // 16 latency ring action_buffer[4][4] (buf_size rows used)
    F_BIAS = 40,        // 3  gyro bias (SensorNoise.gyro_bias)
    F_LPF = 43,         // 3  gyro low-pass filter state
    F_HELD = 46,        // 10 held 100 Hz measurement (xyz, quat, vel); persistent only if agg % obs_rate
    F_OBS_PREV = 56,    // 17 previous observation o_{k-1} (13 used with noise)
    F_HIST_ACT = 73,    // 8  action_history [2][4]
    F_PARAM = 81,       // 19 per-env DR params: dt, m, Jx, Jy, Jz, k0, k1, A[4], B[4], K[4]
    F_DSTB = 100,       // 3  per-episode / current-gust disturbance torque
    F_LEVEL = 103,      // 1  disturbance level of the episode
    F_MOTOR_LO = 104,   // 4  low word of the motor state (x + x_lo, compensated recurrence)
    NF = 108
};
// ---- int state fields ----
enum : int {
    I_EP_STEP = 0,      // env-steps since reset (TimeLimit, iteration = ep_step * agg)
    I_RNG = 1,          // Philox counter (one per env-step / reset)
    I_FLAGS = 2,        // bits 0-3 action_idx, 4-5 action_history alias bits, 6 last_action alias,
                        // 7 a physics sub-step ran since the reset (prop joints spin)
    I_LEVEL = 3,        // Boltzmann level index / HJ table row
    I_GUST = 4,         // env-steps left in the current gust
    NI = 5
};
enum { NUM_PARAMS = 19 };

// ---- internal state layout (what the kernels read and write) ----
// AoSoA of float4 groups: tiles of 64 envs (one wave); inside a tile, group g of lane l is the
// 16 B at tile_base + g * 1024 + l * 16.  Every state access is a coalesced dwordx4 (1 KB per
// wave instruction).  Int fields live in the same array as bit patterns.  Groups are arranged
// so that a config touches whole groups: read-write state, read-only per-episode parameters and
// optional fields never share a group.  The public snapshot format of cf2_get_state /
// cf2_set_state stays the plain SoA above (F_* / I_* fields); conversion kernels map it.
enum : int {
    S_POS = 0, S_QUAT = 3, S_VEL = 7, S_OMEGA = 10,      // G0-G3 (always read + written)
    S_EP = 13, S_RNG = 14, S_FLAGS = 15,                  //   ints in G3
    S_MOTOR = 16,                                         // G4
    S_OU = 20,                                            // G5
    S_ABUF = 24,                                          // G6-G9, row r in G6+r
    S_BIAS = 40, S_GUST = 43,                             // G10: gyro bias + gust_left (int)
    S_LPF = 77,                                           // G19.yzw, sensor noise only (G19.x = obs_prev[12]);
                                                          //   G11 is unused
    S_RPY = 48,                                           // G12 (Simple physics)
    S_DSTB = 52,                                          // G13
    S_HACT = 56,                                          // G14-G15
    S_OBSP = 64,                                          // G16-G20 (13 or 17 used)
    S_HELD = 84,                                          // G21-G23 (held_persistent only)
    S_PARAM = 96,                                         // G24-G27.z: 15 DR params (dt, m, J, k0, k1,
                                                          //   B[4], K[4]; A = 1 - B is not stored)
    S_LEVEL = 111,                                        // G27.w
    S_MOTOR_LO = 112,                                     // G28: motor-state low words
    S_LEVEL_IDX = 116,                                    // G29.x (int)
    NS = 120, NG = 30
};
__host__ __device__ constexpr uint32_t tiles_of(uint32_t n) { return (n + 63u) / 64u; }
__host__ __device__ constexpr size_t state_bytes(uint32_t n) { return (size_t)tiles_of(n) * NG * 1024u; }
enum { HJ_PTS = 15, HJ_TABLE = 11390625 };
// up to this many envs per context the env kernels run 64 envs per 256-thread block with helper
// waves (step_kernel_small, rollout_kernel_small, collect_kernel_small)
constexpr uint32_t SMALL_N_MAX = 32768;
enum { PHYS_BULLET_T = 0, PHYS_SIMPLE_T = 1 };
enum { DSTB_NONE_T = 0, DSTB_EXTERNAL_T = 1, DSTB_UNIFORM_T = 2, DSTB_CONST_T = 3, DSTB_GUST_T = 4, DSTB_HJ_T = 5 };
enum { LEVEL_FIXED_T = 0, LEVEL_BOLTZMANN_T = 1 };
enum : uint32_t { TAG_STEP = 1, TAG_RESET = 2, TAG_PHYS = 3 };

// Kernel parameter block, passed by value (kernarg segment -> scalar loads).
struct KParams {
    uint32_t N, gid_off, key0, key1;
    uint32_t late_block;          // step kernel: first block index past one residency round (set per launch)
    uint32_t out_stride;          // rollout kernel: rows per per-step output slab (set per launch)
    // host-side, set once at cf2_create for the context's device and configuration: blocks
    // resident at once of the large-N step / fused rollout / fused collect kernels and of the
    // small-N collect rollout kernel (query_occupancy), and whether the step's working set exceeds the Infinity Cache
    // (nt state stores)
    uint32_t rb_step, rb_roll, rb_collect, rb_croll_small, nt_state;
    int32_t agg, obs_rate, buf_size, use_latency, use_motor_dyn, max_steps, auto_reset, reset_dist;
    int32_t dstb_mode, level_mode, num_levels, gust_dur, noise, dr, phys, held_persistent, need_level;
    float time_step, mass, ixx, iyy, izz, ft0, ft1, K, A, B, hover_x, hover_action, ou_sigma;
    float drag_xy, drag_z, g_world, g_agent, arm, prop_xy, prop_z, prop_mass, prop_inertia, prop_speed_gain;
    float lin_damping, ang_damping, vmax;
    float init_xyz[3], pos_lim, angle_lim, yaw_lim, vel_lim, rate_lim, yaw_rate_lim, action_std, motor_std;
    float dr_lo[9], dr_hi[9];     // dt, m, Jx, Jy, Jz, k0, k1, mtc, t2w
    float pos_std, pos_unif, vel_std, rot_std, rot_unif, pgd, sbgd, gyro_rw, gyro_ton, lpf_gain, lpf_ratio;
    float pen_action, pen_angle, pen_spin, pen_term, pen_vel, pen_z, pen_arp, pen_dist;
    float target_pos[3], target_rpy[3], target_rate[3];
    float done_rp, done_rate_deg, done_zmin, cost_xy, cost_z, cost_rp, cost_vel, cost_rate;
    float level_fixed, umax[3], gust_p, gust_max;
    double umax_d[3], uni_hi[3];
    int32_t num_drones, downwash_on;                  // multi-drone formations (f4)
    float dw_coeff[3], prop_radius, formation_dx, formation_dz;
    int32_t ground_effect;                            // BasePhysics.use_ground_effect (physics.py:18-25)
    float gnd_eff_coeff, gnd_eff_h_clip;
    const struct KTables* tab;   // device-resident lookup tables (dynamically indexed)
    const float* V;              // HJ value tables [num_tables][15^6]
    const uint8_t* hj_bits;      // per-node disturbance sign bits of V [num_tables][15^6] (cf2_bind_hj_tables)
};

// Lookup tables indexed with per-env (divergent) indices: kept in device memory, not in the
// kernarg block (a dynamically indexed by-value kernel argument is copied to scratch).
struct KTables {
    double level_cdf[32];
    float level_values[32];
    int32_t table_of_level[32];
    double hj_grid[6][HJ_PTS];
    // reset-only parameters (copies of the KParams fields of the same names): read by the reset
    // code from here, so the step's kernarg block loads ~35 fewer scalars at kernel entry
    float init_xyz[3], pos_lim, angle_lim, yaw_lim, vel_lim, rate_lim, yaw_rate_lim;
    float action_std, motor_std, hover_x, hover_action;
    float dr_lo[9], dr_hi[9];
    uint32_t dev_err;           // CF2_DEVERR_* bits the kernels set (cf2_device_errors); 0 when uploaded
};
enum : uint32_t { CF2_DEVERR_HANDOVER = 1u };   // a helper wave gave up waiting for an LDS hand-over

struct StepIO {
    float* sf;          // internal AoSoA state (state_bytes(N))
    const float* act;
    const float* dstb;
    float* obs;
    float* rew;
    uint8_t* done;
    uint8_t* trunc;
    float* cost;
    float* level;
    float* final_obs;
};

// records e as the thread's last HIP error (cf2_last_hip_error) and maps it to a cf2_status
int hip_fail(hipError_t e);
// fills P.rb_* for the kernel instances P dispatches to, on the current device
hipError_t query_occupancy(KParams& P);
hipError_t launch_step(const KParams& P, const StepIO& io, hipStream_t s);
// the env-step with the delta exchange's pack of its observations fused in (the step kernels'
// epilogues)
hipError_t launch_step_packed(const KParams& P, const StepIO& io, const PackIO& pio, hipStream_t s);
// The collect loop's policy half, fused behind the env-step (collect_kernel): the actor-critic
// forward on the new observations (packed bf16x3 fragments of cf2_policy_pack, obs_dim 34)
struct PolicyIO {
    const float* w;                 // packed fragments
    uint32_t key0, key1, counter;   // sampling noise: Philox(seed, counter, row_offset + row)
    uint32_t row_offset;
    float* act;                     // [N, 4] sampled actions for the next env-step
    float* val;                     // [N] V(obs)
    float* logp;                    // [N] log-probabilities of act
};
// returns hipErrorNotSupported when the config has no fused instance (the caller then launches
// cf2_step and cf2_policy_forward)
hipError_t launch_collect(const KParams& P, const StepIO& io, const PolicyIO& pio, hipStream_t s);
// K steps of the collect loop in one launch (collect_rollout_kernel): env-step k reads the actions
// at pio.act + k * N * 4 and writes io's k-th [N, ...] slabs (obs, rew, done, trunc, final_obs);
// the policy on its observations writes slab k + 1 of pio.act / pio.val / pio.logp ([K + 1][N]),
// noise counter pio.counter + k.  hipErrorNotSupported where collect_kernel has no instance.
hipError_t launch_collect_rollout(const KParams& P, const StepIO& io, const PolicyIO& pio, uint32_t K, hipStream_t s);
// K fused env-steps (state in registers); outputs [K][N][...] slabs, actions at act + k * act_stride
hipError_t launch_rollout(const KParams& P, const StepIO& io, uint32_t K, uint32_t act_stride, hipStream_t s);
hipError_t launch_reset(const KParams& P, float* sf, const uint8_t* mask, float* obs, hipStream_t s);
hipError_t launch_init(const KParams& P, float* sf, hipStream_t s);
// one physics sub-step of every env (physics plugin step_forward); dt_override <= 0: per-env dt
hipError_t launch_physics(const KParams& P, float* sf, const float* act, const float* dstb, float dt_override,
                          hipStream_t s);
// public SoA snapshot <-> internal AoSoA (to_public = 1: internal -> state_f/state_i)
hipError_t launch_state_convert(const KParams& P, float* sf, float* state_f, int32_t* state_i, int to_public,
                                hipStream_t s);
struct HjGrid { double p[6][HJ_PTS]; };   // grid nodes by value (hj_kernel kernarg)
hipError_t launch_hj(const HjGrid& G, const double umax[3], const float* V, const float* states, uint32_t n,
                     float level, float* dstb, float* uopt, hipStream_t s);
// the sign bits hj_signs derives from the 7 taps around each grid node, for every node of every table
hipError_t launch_hj_sign_table(const float* V, uint32_t num_tables, uint8_t* bits, hipStream_t s);

}  // namespace cf2
