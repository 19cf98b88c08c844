/*
 * cf2sim.h -- C ABI of the MI355X-native batched CrazyFlie hover environment.
 *
 * One context owns N independent hover environments whose state lives in HBM as
 * structure-of-arrays.  Every entry point is asynchronous on the caller's HIP stream;
 * every I/O buffer is a caller-owned DEVICE pointer.  Return value: 0 on success or a
 * negative cf2_status; the library never aborts the process.
 *
 * Reference interfaces replaced (paths relative to the reference repository root,
 * phoenix_drone_simulation/ omitted):
 *   cf2_reset  <- DroneBaseEnv.reset                         envs/base.py:420-464
 *                 + task_specific_reset                       envs/hover_free.py:237-289, envs/hover.py:204-256
 *                 + apply_domain_randomization                envs/base.py:241-298
 *                 + RandomHJ level redraw (Boltzmann)         envs/hover_free.py:492-536, envs/utils.py:27-39
 *   cf2_step   <- DroneBaseEnv.step and its adversary overrides
 *                                                             envs/base.py:466-507, envs/hover_free.py:391-444,
 *                                                             :778-835, :950-1007; envs/hover.py:649-702, ...
 *                 (one call = aggregate_phy_steps x PybulletPhysicsWithAdversary.step_forward
 *                  envs/physics.py:213-250 / PyBulletPhysics.step_forward :91-124 /
 *                  SimplePhysics.step_forward :130-200, then compute_history/reward/info/done,
 *                  then gym TimeLimit(max_episode_steps) and auto-reset)
 *   cf2_hj_disturbance <- distur_gener                        adversarial_generation/FasTrack_data/distur_gener.py:19-183
 *                         (+ Grid.get_index                   adversarial_generation/odp/Grid/GridProcessing.py:52-71)
 *   cf2_get_state / cf2_set_state: SoA snapshot (the reference never checkpoints env state;
 *                 used for parity tests and checkpoint/resume of rollouts).
 */
#ifndef CF2SIM_H
#define CF2SIM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CF2SIM_ABI_VERSION 8

typedef enum cf2_status {
    CF2_OK = 0,
    CF2_ERR_INVALID_ARG = -1,   /* null pointer, bad enum, inconsistent sizes */
    CF2_ERR_OUT_OF_MEMORY = -2, /* hipMalloc failed */
    CF2_ERR_HIP = -3,           /* a HIP runtime call failed (see cf2_last_hip_error) */
    CF2_ERR_UNSUPPORTED = -4,   /* configuration outside what the kernels implement */
    CF2_ERR_NO_TABLE = -5       /* HJ disturbance requested but no value table bound */
} cf2_status;

/* physics plugin (envs/physics.py) */
enum { CF2_PHYS_BULLET = 0,   /* PyBulletPhysics / PybulletPhysicsWithAdversary: rigid-body restatement of the
                                 btMultiBody step (bullet3 3.21) the reference delegates to stepSimulation() */
       CF2_PHYS_SIMPLE = 1 }; /* SimplePhysics: explicit Euler on rpy (envs/physics.py:130-200) */

/* task (reward / done / reset flavour) */
enum { CF2_TASK_HOVER = 0,       /* DroneHoverBaseEnv  envs/hover.py:16-256 */
       CF2_TASK_HOVER_FREE = 1 };/* DroneHoverFreeEnv  envs/hover_free.py:17-289 */

/* disturbance source (the dstb argument of PybulletPhysicsWithAdversary.step_forward) */
enum { CF2_DSTB_NONE = 0,      /* dstb = (0,0,0)                       hover_free.py:814 */
       CF2_DSTB_EXTERNAL = 1,  /* caller passes dstb[N,3] each step     (test / custom adversary hook) */
       CF2_DSTB_UNIFORM = 2,   /* dstb_space.sample() each env-step    hover_free.py:986, hover.py:1244 */
       CF2_DSTB_CONST = 3,     /* per-episode constant torque ("constant wind", BASELINE config 2) */
       CF2_DSTB_GUST = 4,      /* Philox-driven torque bursts (BASELINE config 4, build-defined) */
       CF2_DSTB_HJ = 5 };      /* HJ bang-bang disturbance from a 15^6 value table  distur_gener.py:19-183 */

/* how the per-episode disturbance level is chosen (HJ / const / gust magnitudes) */
enum { CF2_LEVEL_FIXED = 0,      /* env.disturbance_level constant, e.g. 1.5 (hover_free.py:319) */
       CF2_LEVEL_BOLTZMANN = 1 };/* Boltzmann() redraw at the end of every reset (hover_free.py:536) */

/* 8 Mi envs per context: the state SoA (104 x 4 B x N) must stay addressable by one 32-bit
   buffer-descriptor range; shard larger populations over several contexts / GPUs. */
#define CF2_MAX_ENVS_PER_CTX  (1u << 23)
#define CF2_HJ_PTS 15               /* grid points per dimension, distur_gener.py:179 */
#define CF2_NUM_LEVELS_MAX 32

typedef struct cf2_config {
    /* ---- sizes / plumbing ---- */
    uint32_t num_envs;             /* envs owned by this context (this rank's shard)             */
    uint32_t env_id_offset;        /* global id of env 0 (rank shard offset): RNG keys use global ids */
    uint64_t seed;                 /* Philox4x32-10 key                                            */

    /* ---- env flavour ---- */
    int32_t physics;               /* CF2_PHYS_*                                                   */
    int32_t task;                  /* CF2_TASK_*                                                   */
    int32_t disturbance;           /* CF2_DSTB_*                                                   */
    int32_t level_mode;            /* CF2_LEVEL_*                                                  */
    int32_t aggregate_phy_steps;   /* physics sub-steps per env-step (2)       base.py:35          */
    int32_t obs_rate;              /* sim_freq // observation_frequency (2)    base.py:106          */
    int32_t buf_size;              /* latency ring length int(latency//dt) (2) agents.py:180        */
    int32_t use_latency;           /* agents.py:165                                                */
    int32_t use_motor_dynamics;    /* agents.py:196                                                */
    int32_t max_episode_steps;     /* gym TimeLimit (500)  __init__.py; 0 = none                    */
    int32_t auto_reset;            /* reset envs on done/truncation inside cf2_step                 */
    int32_t enable_reset_distribution; /* base.py:38                                                */
    int32_t observation_noise_on;  /* observation_noise > 0                    hover_free.py:170    */
    int32_t domain_randomization_on; /* domain_randomization > 0               base.py:261          */
    double  domain_randomization;  /* DR factor (0.10)                                              */
    double  motor_thrust_noise;    /* OU sigma = 0.2 * this                    agents.py:206        */

    /* ---- time ---- */
    double sim_freq;               /* Hz (200 bullet, 100 simple)                                  */
    double time_step;              /* 1/sim_freq (nominal; DR redraws per env)                      */

    /* ---- robot constants (URDF + agents.py:142-206) ---- */
    double mass, arm, thrust2weight, ixx, iyy, izz;
    double drag_xy, drag_z;
    double gravity_agent;          /* 9.81  agents.py:145 (K formula)          */
    double gravity_world;          /* 9.81  bc.setGravity base.py:192 / SimplePhysics G physics.py:16 */
    double motor_time_constant;    /* 0.080 */
    double ft0, ft1;               /* FORCE_TORQUE_FACTOR_0/1  agents.py:142-143 */
    double K, A, B;                /* nominal MAX_THRUST, 1 - Ts/T, Ts/T */
    double hover_x, hover_action;  /* sqrt(1/t2w), 2/t2w - 1 */
    double prop_mass, prop_inertia;/* cf21x_bullet.urdf m1..m4_link: 1e-9 kg, 1e-9 kg m^2 */
    double prop_xy, prop_z;        /* prop joint origins (+-0.028, +-0.028, 0.0108) */
    double prop_speed_gain;        /* setJointMotorControl2 targetVelocity = x*100  agents.py:327 */
    double lin_damping, ang_damping;   /* btMultiBody default 0.04 / 0.04 */
    double max_coord_velocity;     /* btMultiBody m_maxCoordinateVelocity 100 */

    /* ---- initial state / reset distribution (hover_free.py:237-289) ---- */
    double init_xyz[3];
    double reset_pos_lim, reset_angle_lim, reset_yaw_lim, reset_vel_lim, reset_rate_lim, reset_yaw_rate_lim;
    double action_init_std, motor_init_std;   /* 0.02, 0.02 */

    /* ---- sensor noise (envs/sensors.py:17-134) & gyro LPF (base.py:107) ---- */
    double pos_norm_std, pos_unif_range, vel_norm_std, vel_unif_range;
    double rot_norm_std, rot_unif_range;
    double gyro_noise_density, gyro_random_walk, gyro_bias_corr_time, gyro_turn_on_bias_sigma;
    double lpf_gain, lpf_ratio;    /* K, T_s/T */

    /* ---- reward / done / cost (hover.py:102-202, hover_free.py:124-235,449-461) ---- */
    double penalty_action, penalty_angle, penalty_spin, penalty_terminal, penalty_velocity, penalty_z;
    double penalty_arp;            /* self.ARP */
    double penalty_dist;           /* 1 for DroneHoverBaseEnv (-dist term), 0 for free */
    double target_pos[3], target_rpy[3], target_rate[3];
    double done_rp_limit;          /* rad: deg2rad(60) or deg2rad(75) */
    double done_rate_limit_deg;    /* 300 or 1000 */
    double done_z_min;             /* 0.2 */
    double cost_xy_lim, cost_z_lim, cost_rp_lim, cost_vel_lim, cost_rate_lim;

    /* ---- disturbance ---- */
    double dstb_level;             /* fixed level (CF2_LEVEL_FIXED) */
    double dstb_umax[3];           /* 5.3e-3, 5.3e-3, 1.43e-4   distur_gener.py:152 */
    double dstb_uniform_hi[3];     /* 1e-3, 1e-3, 1e-4          hover_free.py:315 */
    double gust_onset_prob, gust_max_level;   /* 0.01, 1.5 */
    int32_t gust_duration;         /* 20 env-steps */
    int32_t num_levels;            /* Boltzmann support size (21) */
    double level_values[CF2_NUM_LEVELS_MAX];  /* np.around(energies, 1) */
    double level_cdf[CF2_NUM_LEVELS_MAX];     /* normalised cumsum(p), numpy choice()  */
    double hj_grid_min[6];         /* per-dim lower bounds (Grid.min)                */
    double hj_grid_dx[6];          /* Grid.dx                                       */
    double hj_grid_points[6][CF2_HJ_PTS]; /* np.linspace node values (Grid.grid_points) */

    /* ---- multi-drone envs (BASELINE config 5; no reference code) ----
     * num_drones consecutive envs form one env group of drones flying a formation: drone k sits at
     * init_xyz + ((k/2 - (ceil(num_drones/2)-1)/2) * formation_dx, 0, (k%2) * formation_dz).
     * downwash_on: each drone feels, from every drone j of its group above it (dz > 0, dxy < 10),
     * the downwash force of gym-pybullet-drones BaseAviary._downwash with the URDF coefficients
     * parsed but unused by the reference (agents.py:251-257):
     *   F = dw_coeff_1 (prop_radius / (4 dz))^2 exp(-0.5 (dxy / (dw_coeff_2 dz + dw_coeff_3))^2)
     * along -z of the body (LINK_FRAME), at the centre of mass.  Bullet physics only. */
    int32_t num_drones;            /* 1 (default), 2, 4 or 8; num_envs and env_id_offset multiples of it */
    int32_t downwash_on;
    double dw_coeff[3];            /* 2267.18, 0.16, -0.11 */
    double prop_radius;            /* 2.31348e-2 m */
    double formation_dx, formation_dz;   /* 0.5 m, 1.0 m */

    /* ---- ground effect (BasePhysics.calculate_ground_effect envs/physics.py:27-58, applied in
     * step_forward physics.py:116-120 / 243-246; the reference's envs never enable it;
     * cf2_physics_step only, see cf2_set_ground_effect): while
     * |roll|, |pitch| < pi/2 each prop gets the extra thrust f_i * gnd_eff_coeff *
     * (prop_radius / (4 max(z_i, gnd_eff_h_clip)))^2, z_i = world height of prop i.  Bullet only. */
    int32_t use_ground_effect;
    double gnd_eff_coeff;          /* URDF gnd_eff_coeff 11.36859 */
    double gnd_eff_h_clip;         /* GND_EFF_H_CLIP agents.py:156 */
} cf2_config;

/* SoA layout descriptor returned by cf2_layout(): state_f[field*num_envs + env],
 * state_i[field*num_envs + env]. Field meaning is documented in DESIGN.md. */
typedef struct cf2_layout {
    uint32_t num_envs;
    uint32_t num_float_fields;
    uint32_t num_int_fields;
    uint32_t obs_dim;              /* 34 with observation noise, 42 without */
    uint32_t obs_len;              /* 13 or 17 */
    uint32_t f_pos, f_quat, f_vel, f_omega, f_rpy, f_motor, f_ou, f_abuf, f_bias, f_lpf, f_held,
             f_obs_prev, f_hist_act, f_param, f_dstb;
    uint32_t i_ep_step, i_rng, i_flags, i_level, i_gust;
    uint32_t num_params;           /* per-env DR parameters (19; the motor A[4] = 1 - B[4] is derived) */
    uint32_t f_motor_lo;           /* 4: low words of the motor state (state = f_motor + f_motor_lo) */
} cf2_layout;

typedef struct cf2_ctx cf2_ctx;

int  cf2_abi_version(void);
/* Errors the kernels of ctx recorded on the device (synchronises the device): bit 1 = a helper
 * wave of the small-N kernels gave up waiting for the LDS hand-over of the reset pose (its reset
 * rows would be built from a stale pose; never observed).  clear != 0 resets the word.  The
 * kernels never trap: they record and finish, and the host decides. */
int  cf2_device_errors(cf2_ctx* ctx, uint32_t* flags_out, int clear);
size_t cf2_config_sizeof(void);     /* lets FFI callers check their struct mirror */
const char* cf2_status_string(int status);
int  cf2_last_hip_error(void);

int  cf2_create(const cf2_config* cfg, cf2_ctx** out_ctx);
int  cf2_destroy(cf2_ctx* ctx);
int  cf2_layout_get(const cf2_ctx* ctx, cf2_layout* out);

/* Bind HJ value tables: V_dev = [num_tables][15^6] float32 C-order [roll,pitch,yaw,p,q,r]
 * (the on-disk fastrack_{level}_15x15.npy format).  table_level_index maps Boltzmann level
 * index -> table row (or -1 = no table, dstb 0).  Caller owns V_dev for the ctx lifetime.
 * Binding derives, once, the disturbance sign bits of every grid node (the distur_gener rule over
 * the node's 7 value taps, distur_gener.py:155-183; 1 byte per node, 11.4 MB per table, owned by
 * the ctx): the env-step gathers one byte per env.  Rebind after changing the table contents.
 * Synchronous and device-wide: waits for all work on the device first (V_dev may have been
 * written on any stream; steps in flight may still read the previous tables), then derives the
 * bits.  On failure the ctx keeps its previous binding, or has none (CF2_ERR_NO_TABLE on the
 * next HJ step) if the previous bits were already overwritten.  num_tables * 15^6 must fit in
 * 32 bits (at most 377 tables). */
int  cf2_bind_hj_tables(cf2_ctx* ctx, const float* V_dev, int num_tables,
                        const int32_t* table_of_level /* host, num_levels entries */);

/* Reset envs whose mask byte is non-zero (mask_dev NULL = all), write their obs rows. */
int  cf2_reset(cf2_ctx* ctx, const uint8_t* mask_dev, float* obs_dev, void* stream);

/* One env-step for all envs.  act_dev [N,4] (16-B aligned); dstb_dev [N,3] (only for CF2_DSTB_EXTERNAL,
 * else NULL); obs_dev [N,obs_dim] (16-B aligned); rew_dev [N]; done_dev [N] (terminal OR truncated, gym 4-tuple semantics);
 * trunc_dev [N] (TimeLimit truncation, may be NULL); cost_dev [N] (may be NULL);
 * level_dev [N] disturbance level of the finished step (may be NULL);
 * final_obs_dev [N,obs_dim] pre-reset observation of envs that auto-reset this step (may be NULL). */
int  cf2_step(cf2_ctx* ctx, const float* act_dev, const float* dstb_dev,
              float* obs_dev, float* rew_dev, uint8_t* done_dev, uint8_t* trunc_dev,
              float* cost_dev, float* level_dev, float* final_obs_dev, void* stream);

/* One physics sub-step of every env, without the env-step around it: the physics plugin's
 * step_forward (PyBulletPhysics.step_forward physics.py:91-124, SimplePhysics :130-200,
 * PybulletPhysicsWithAdversary.step_forward :213-250; plugin construction envs/base.py:223-232):
 * apply_action (latency ring, PWM, OU thrust noise, motor dynamics), motor forces + yaw torque,
 * adversary torques dstb[0], dstb[1] (dstb_dev [N,3] or NULL = none), drag, the rigid-body step
 * and update_information.  No observation, reward, TimeLimit or auto-reset.  time_step > 0
 * overrides every env's dt for this call (BasePhysics.set_parameters physics.py:60-68); <= 0
 * uses the per-env dt (domain randomisation).  act_dev [N,4] 16-B aligned. */
int  cf2_physics_step(cf2_ctx* ctx, const float* act_dev, const float* dstb_dev, float time_step, void* stream);
/* Ground effect on / off for this context's Bullet physics (the physics object's
 * use_ground_effect, envs/physics.py:18-25); the initial value is cfg.use_ground_effect.
 * It applies to cf2_physics_step only: the reference's envs build their physics with the default
 * use_ground_effect=False (envs/base.py:223-232), so the env-step kernels carry no ground-effect
 * code and cf2_step / cf2_rollout return CF2_ERR_UNSUPPORTED while it is on.
 * Returns CF2_ERR_UNSUPPORTED for SimplePhysics contexts. */
int  cf2_set_ground_effect(cf2_ctx* ctx, int on);

/* K consecutive env-steps fused in one launch (rollout mode; SURVEY section 7 "fused K-step"):
 * the env state stays in registers across the K steps.  Step k reads actions act_dev + k *
 * act_stride_elems ([N,4], 16-B aligned, stride a multiple of 4) and writes the k-th [N, ...]
 * slab of every output: obs_dev [K,N,obs_dim] (8-B aligned), rew_dev [K,N], done_dev [K,N] and,
 * when not NULL, trunc_dev [K,N], cost_dev [K,N], level_dev [K,N], final_obs_dev [K,N,obs_dim].
 * Results are identical to K cf2_step calls with the same actions (the reference's
 * IWPGAlgorithm.roll_out loop algs/iwpg/iwpg.py:372-410 with actions known in advance, e.g.
 * open-loop or random-action rollouts).  Not for CF2_DSTB_EXTERNAL envs (CF2_ERR_UNSUPPORTED). */
int  cf2_rollout(cf2_ctx* ctx, int K, const float* act_dev, size_t act_stride_elems,
                 float* obs_dev, float* rew_dev, uint8_t* done_dev, uint8_t* trunc_dev,
                 float* cost_dev, float* level_dev, float* final_obs_dev, void* stream);

/* Whole-state snapshot (device buffers sized by cf2_layout). */
int  cf2_get_state(const cf2_ctx* ctx, float* state_f_dev, int32_t* state_i_dev, void* stream);
int  cf2_set_state(cf2_ctx* ctx, const float* state_f_dev, const int32_t* state_i_dev, void* stream);

/* Stand-alone batched distur_gener: states_dev [n,6] = [roll,pitch,yaw,p,q,r] (float32),
 * V_dev one 15^6 table, out dstb_dev [n,3] = opt_d, out uopt_dev [n,3] = opt_u (may be NULL). */
int  cf2_hj_disturbance(const cf2_config* cfg, const float* V_dev, const float* states_dev,
                        uint32_t n, float level, float* dstb_dev, float* uopt_dev, void* stream);

/* ---- batched rollout caller ----
 * Gaussian MLP actor-critic forward of the reference's PPO networks for a batch of observations,
 * one fused launch on the matrix cores: ActorCritic.step (algs/core.py:371-395), MLPGaussianActor
 * (core.py:228-291) pi D->50->50->4 ReLU, MLPCritic D->64->64->1 tanh (algs/ppo/defaults.py:8-13).
 * fp32 activations and accumulation; products in one of two precisions:
 *   CF2_POLICY_F32     exact fp32 (v_mfma_f32_16x16x4_f32, the result of an fmaf chain over k);
 *   CF2_POLICY_BF16X3  split-bf16 operands (x = hi + lo, three bf16 MFMAs per product block):
 *                      <= ~1.1e-5 relative error per product, ~5x the fp32 rate.
 * Weights: the flat block (cf2_policy_weights_count(D) floats; layout in csrc/cf2sim_policy.hip:
 * input-major matrices, pi then v, log_std after the pi head) is converted once per weight update
 * by cf2_policy_pack into the packed block (cf2_policy_packed_count(D, precision) floats, 16-B
 * aligned: MFMA operand fragments in the kernel's order) that the forward calls take with the
 * same precision.
 * obs_dev [n, D] (D = 34 or 42, 8-B aligned); sample != 0: act = mu + exp(log_std) * eps,
 * eps ~ N(0,1) from Philox keyed (seed, counter, row + row_offset); else act = mu.  Outputs
 * act_dev [n,4] (16-B aligned), val_dev [n], logp_dev [n] (sum of Normal log-densities; may be
 * NULL). */
enum cf2_policy_precision { CF2_POLICY_F32 = 0, CF2_POLICY_BF16X3 = 1 };
size_t cf2_policy_weights_count(uint32_t obs_dim);
size_t cf2_policy_packed_count(uint32_t obs_dim, int precision);
int  cf2_policy_pack(const float* weights_dev, uint32_t obs_dim, int precision, float* packed_dev, void* stream);
int  cf2_policy_forward(const float* packed_dev, uint32_t n, uint32_t obs_dim, int precision, const float* obs_dev,
                        uint64_t seed, uint32_t counter, uint32_t row_offset, int sample,
                        float* act_dev, float* val_dev, float* logp_dev, void* stream);
/* Value of the rows with mask_dev[r] != 0 only (time-out bootstraps V(final obs)); other rows of
 * val_dev are left untouched. */
int  cf2_value_forward_masked(const float* packed_dev, uint32_t n, uint32_t obs_dim, int precision,
                              const float* obs_dev, const uint8_t* mask_dev, float* val_dev, void* stream);

/* One step of the collect loop in one launch: the env-step of cf2_step (act_dev -> obs_dev, rew,
 * done, trunc, final_obs; same arguments, no disturbance tensor, no cost/level outputs), then
 * cf2_policy_forward(sample = 1) on the new observations -> act_out_dev [N,4] (16-B aligned, the
 * next env-step's actions; must not be act_dev), val_out_dev [N], logp_out_dev [N].  Replaces the
 * pair env.step + ac.step of IWPGAlgorithm.roll_out (phoenix_drone_simulation/algs/iwpg/iwpg.py:
 * 377-380; ActorCritic.step algs/core.py:371-395).  Every output is bit-identical to the two
 * calls.  Fused only where built (precision CF2_POLICY_BF16X3, obs_dim 34 = sensor noise on, the
 * default Bullet env-step shape, one drone per formation; any N); elsewhere it returns
 * CF2_ERR_UNSUPPORTED and launches nothing, and the caller makes the two calls. */
int  cf2_collect_step(cf2_ctx* ctx, const float* act_dev, float* obs_dev, float* rew_dev, uint8_t* done_dev,
                      uint8_t* trunc_dev, float* final_obs_dev, const float* packed_dev, uint32_t obs_dim,
                      int precision, uint64_t seed, uint32_t counter, uint32_t row_offset, float* act_out_dev,
                      float* val_out_dev, float* logp_out_dev, void* stream);

/* K steps of the collect loop: env-step k (actions act_dev + k*N*4) and then the policy forward +
 * sampling on its observations (noise counter counter + k), whose actions the next env-step
 * takes.  N <= 32768 (C2, the 8-GPU node shard): one launch, the env state in registers for the K
 * steps (64-env groups with helper waves computing the auto-resets, as cf2_step there); larger N:
 * one cf2_collect_step launch per step (faster there than a one-launch loop).  Buffers, slab-major:
 * act_dev [K+1,N,4] (slab 0 in: the first step's actions; slabs 1..K out), val_dev / logp_dev
 * [K+1,N] (slabs 1..K out, slab 0 untouched), obs_dev [K,N,obs_dim] (slab k = the observation
 * after env-step k), rew_dev / done_dev [K,N], trunc_dev / final_obs_dev [K,N] / [K,N,obs_dim]
 * or NULL.  Every output is bit-identical to K cf2_collect_step calls with act_out = the next
 * slab and counters counter, counter + 1, ... (IWPGAlgorithm.roll_out's loop,
 * phoenix_drone_simulation/algs/iwpg/iwpg.py:372-410, ActorCritic.step algs/core.py:371-395).
 * Built where cf2_collect_step is (else CF2_ERR_UNSUPPORTED, nothing launched). */
int  cf2_collect_rollout(cf2_ctx* ctx, int K, float* act_dev, float* obs_dev, float* rew_dev, uint8_t* done_dev,
                         uint8_t* trunc_dev, float* final_obs_dev, const float* packed_dev, uint32_t obs_dim,
                         int precision, uint64_t seed, uint32_t counter, uint32_t row_offset, float* val_dev,
                         float* logp_dev, void* stream);

/* Batched GAE over [T, n] rollout buffers (algs/core.py:459-535 finish_path on every env's
 * episode slices): done/trunc uint8 (terminal -> bootstrap 0, time-out -> trunc_val), the end of
 * the buffer bootstraps last_val [n].  rew_den > 0: reward scaling, delta uses
 * clip(r / rew_den, -10, 10) with rew_den = ret_oms.std + 1e-5 (core.py:522-529); <= 0: none.
 * Outputs adv [T, n], ret = adv + val [T, n] and, if disc_ret_dev is not NULL, the per-episode
 * discounted returns of the unscaled rewards (core.py:519, the return statistics' input). */
int  cf2_gae(uint32_t T, uint32_t n, const float* rew_dev, const float* val_dev, const uint8_t* done_dev,
             const uint8_t* trunc_dev, const float* trunc_val_dev, const float* last_val_dev, float gamma,
             float lam, float rew_den, float* adv_dev, float* ret_dev, float* disc_ret_dev, void* stream);

/* Multi-GPU observation exchange as deltas (the north star's per-step RCCL
 * all-gather of the obs slab).  The reference has no counterpart: its MPI ranks exchange only
 * gradients and statistics (utils/mpi_tools.py:30-44); the rows materialised here are exactly what
 * compute_history (envs/base.py:305-321) returns on every rank.
 * A row is [o_{k-1}, A0, o_k, A1] (obs_len OL = 13 with sensor noise, 17 without); per env-step a
 * rank packs only o_k of every env, a bitmap of the envs that auto-reset and, for up to `cap` of
 * them, the reset row's o_0 and action part, into cf2_obs_packed_words(n, OL, cap) 32-bit words
 * (a multiple of 4).  After an all-gather of the packed buffers ([world][words], rank order,
 * equal shards of n envs) a receiver keeps them and only advances every env's steps since its
 * reset (cf2_obs_consume: age_dev uint16 [world n], saturating; all 0 after the observations came
 * from a full gather right after a reset of every env).  Rows are materialised on request
 * (cf2_obs_rows) from the gathered buffers of step k (capacity cap) and k - 1 (cap_prev), the ages
 * after step k's consume and the actions of steps k, k - 1 and k - 2 (act, act_prev, act_prev2:
 * [world n, 4]); out gets rows [row0, row0 + nrows) as [nrows, 2 OL + 8].  Rank r's packed buffer
 * is at r * stride words (0: cf2_obs_packed_words(n, OL, cap), the all-gather of one step).  Time-out look-ahead:
 * envs whose age becomes watch_age at a consume (max_episode_steps - L; 0xFFFFFFFF: off) are
 * counted per rank into pred_dev[world] (pred_next_dev[world], a different row, is zeroed for the
 * next step): at most that many envs time out L steps later, so the caller can size that step's
 * cap.  Valid under auto-reset for env-step shapes whose action buffer holds only the step's action
 * after a step (aggregate_phy_steps a multiple of buf_size, latency on: the reference's default).
 * Side slots go to 64-env pack blocks, never to single envs (layout and allocation:
 * csrc/cf2sim_pack.h); a block whose resets find no room in the side slab (an overflow) is marked
 * dropped: exactly its reset rows have NaN in their o_0 / A parts, *overflow_dev counts the dropped
 * blocks, every other row and all o_k parts stay exact, and later steps are exact again.  A pack
 * counts spill slots in scratch_dev (PACK_SCRATCH_WORDS = 32 words, zeroed before the pack) and
 * zeroes next_scratch_dev (the counter of the next pack on its stream; or NULL). */
size_t cf2_obs_packed_words(uint32_t n, uint32_t obs_len, uint32_t cap);
int  cf2_obs_pack(const float* obs_dev, const uint8_t* reset_dev, uint32_t n, uint32_t obs_len, uint32_t cap,
                  uint32_t* packed_dev, uint32_t* scratch_dev, uint32_t* next_scratch_dev, void* stream);
/* The env-step (cf2_step's outputs, no final_obs) with the pack of its observations fused in: the
 * env kernel writes packed_dev (cf2_obs_packed_words(N, OL, cap) words) as cf2_obs_pack would, from
 * the rows it has in LDS, so no pack launch re-reads them (step_kernel_small's wave 2 at N <= 32 768,
 * every thread of step_kernel's blocks above), except the 4 informational header words, which it
 * leaves as they are (no receiver reads them).  scratch_dev: this buffer's spill counter
 * (PACK_SCRATCH_WORDS = 32 words), zeroed by the caller before the call (cf2_xchg_* zeroes a
 * batch's counters in the batch's consume, after its packs). */
int  cf2_step_packed(cf2_ctx* ctx, const float* act_dev, float* obs_dev, float* rew_dev, uint8_t* done_dev,
                     uint8_t* trunc_dev, float* cost_dev, float* level_dev, uint32_t* packed_dev, uint32_t* scratch_dev,
                     uint32_t cap, void* stream);
int  cf2_obs_consume(const uint32_t* packed_all_dev, uint32_t world, uint32_t n, uint32_t obs_len, uint32_t cap,
                     uint16_t* age_dev, uint32_t* overflow_dev, uint32_t watch_age, uint32_t* pred_dev,
                     uint32_t* pred_next_dev, void* stream);
int  cf2_obs_rows(const uint32_t* packed_all_dev, uint32_t cap, uint32_t stride, const uint32_t* packed_prev_all_dev,
                  uint32_t cap_prev, uint32_t stride_prev, uint32_t world, uint32_t n, uint32_t obs_len,
                  const uint16_t* age_dev, const float* act_dev, const float* act_prev_dev, const float* act_prev2_dev,
                  uint32_t row0, uint32_t nrows, float* rows_dev, void* stream);

/* The same exchange driven natively: an RCCL communicator of this library's own (one rank per GPU,
 * created on the current device, with an exchange stream of its own) and, per batch of env-steps,
 * one ncclAllGather of the batch's packed buffers and one consume on the exchange stream after the
 * env stream's work so far.  cf2_xchg_bind: the RCCL library to use (NULL: "librccl.so.1"); an
 * instance the process has already loaded (e.g. PyTorch's) is reused.  cf2_xchg_unique_id: on one
 * rank, the 128-byte id every rank passes to cf2_xchg_create (collective: all ranks call it
 * together; depth 2..8 buffer regions).  cf2_xchg_register: the buffers, once: obs [n, 2 OL + 8] /
 * reset uint8 [n] per region (depth each), send (cf2_xchg_send_words, zeroed) and recv
 * (cf2_xchg_recv_words) for batches of up to kmax env-steps, age [world n], overflow, pred (the
 * look-ahead ring [npred][world], used when watch_age is on; npred >= 33).  Every publish / batch
 * takes the next region (0, 1, ..., depth - 1, 0, ...; `region` must name it: the caller keeps the
 * count) and first makes env_stream wait for the all-gather that last read that region.  A batch of
 * nb steps at capacity cap leaves recv region q as [world][nb][cf2_obs_packed_words(n, OL, cap)]:
 * the packed buffer of its step s for rank r at (r * nb + s) * words, i.e. cf2_obs_rows with
 * stride nb * words.
 * cf2_xchg_publish(x, k, cap, region, env_stream): the exchange of env-step k, whose env-step the
 * caller issued on env_stream into obs / reset of `region` (after cf2_xchg_wait_free(x, region,
 * env_stream)); packs it on env_stream, and the exchange runs inline on env_stream too.
 * cf2_xchg_run: env-steps k0 .. k0 + nb - 1 of ctx (nb <=
 * kmax; actions of step k at act_dev[k % nact]) issued back to back on env_stream with their pack
 * fused in (cf2_step_packed), then the batch's exchange at
 * capacity cap; pred_host (pinned, npred x world words, or NULL) receives the look-ahead ring after
 * the batch's consume; the batch's exchange runs on the library's exchange stream (forked from
 * env_stream), so the next batch's env-steps overlap it.  cf2_xchg_env_step: one env-step and its
 * exchange inline on env_stream (no fork, no event: for a consumer that needs every step's rows
 * before it issues the next step; pred_host as for cf2_xchg_run).  Callers on other streams are
 * ordered after inline exchanges by cf2_xchg_wait / wait_free / the next region take.  The same batch with its
 * actions given one env-step at a time (a policy in the loop, acting on each step's local rows):
 * cf2_xchg_begin(x, cap, region, env_stream) opens it (takes the region), cf2_xchg_step(x, ctx, act,
 * rew, trunc, cost, level, env_stream) issues its next env-step (up to kmax), cf2_xchg_end(x, k0,
 * pred_host, env_stream) issues its exchange; cf2_xchg_run is begin + nb steps + end.  cf2_xchg_wait(x, stream): a
 * stream waits until every exchange issued so far is complete.  cf2_xchg_pred_to_host(x, pred_host,
 * stream): the same wait, then the look-ahead ring to pred_host.  Both ring copies are device stores
 * into the pinned buffer's mapping (a kernel on the stream), which never hold the calling thread;
 * memory that is not mapped pinned memory falls back to hipMemcpyAsync.  RCCL failures return
 * CF2_ERR_HIP. */
typedef struct cf2_xchg cf2_xchg;
int  cf2_xchg_bind(const char* rccl_path);
int  cf2_xchg_unique_id(uint8_t* id_out, size_t id_len);
int  cf2_xchg_create(const uint8_t* id, size_t id_len, uint32_t world, uint32_t rank, uint32_t depth,
                     cf2_xchg** out);
int  cf2_xchg_destroy(cf2_xchg* x);
size_t cf2_xchg_send_words(uint32_t n, uint32_t obs_len, uint32_t depth, uint32_t kmax);
size_t cf2_xchg_recv_words(uint32_t n, uint32_t obs_len, uint32_t world, uint32_t depth, uint32_t kmax);
int  cf2_xchg_register(cf2_xchg* x, uint32_t n, uint32_t obs_len, uint32_t watch_age, uint32_t kmax,
                       float* const* obs_dev, uint8_t* const* reset_dev, uint32_t* send_dev, uint32_t* recv_dev,
                       uint16_t* age_dev, uint32_t* overflow_dev, uint32_t* pred_dev, uint32_t npred);
int  cf2_xchg_publish(cf2_xchg* x, uint64_t k, uint32_t cap, uint32_t region, void* env_stream);
int  cf2_xchg_wait_free(cf2_xchg* x, uint32_t region, void* stream);
int  cf2_xchg_wait(cf2_xchg* x, void* stream);
int  cf2_xchg_pred_to_host(cf2_xchg* x, uint32_t* pred_host, void* stream);
int  cf2_xchg_run(cf2_xchg* x, cf2_ctx* ctx, uint64_t k0, uint32_t nb, uint32_t cap, uint32_t region,
                  const float* const* act_dev, uint32_t nact, float* rew_dev, uint8_t* trunc_dev, float* cost_dev,
                  float* level_dev, uint32_t* pred_host, void* env_stream);
int  cf2_xchg_begin(cf2_xchg* x, uint32_t cap, uint32_t region, void* env_stream);
int  cf2_xchg_step(cf2_xchg* x, cf2_ctx* ctx, const float* act_dev, float* rew_dev, uint8_t* trunc_dev, float* cost_dev,
                   float* level_dev, void* env_stream);
int  cf2_xchg_end(cf2_xchg* x, uint64_t k0, uint32_t* pred_host, void* env_stream);
int  cf2_xchg_env_step(cf2_xchg* x, cf2_ctx* ctx, uint64_t k, uint32_t cap, uint32_t region, const float* act_dev,
                       float* rew_dev, uint8_t* trunc_dev, float* cost_dev, float* level_dev, uint32_t* pred_host,
                       void* env_stream);
/* cf2_xchg_copy_sync: the host waits for the latest look-ahead count copy into pred_host (a buffer
 * an exchange of cf2_xchg_run / cf2_xchg_end was given; up to 64 distinct buffers per exchange);
 * CF2_ERR_INVALID_ARG for a buffer no exchange copied into. */
int  cf2_xchg_copy_sync(cf2_xchg* x, const uint32_t* pred_host);
/* Diagnostics (no reference counterpart): host time of the exchange's C calls by part, ns summed
 * over the cf2_xchg_run / cf2_xchg_env_step calls counted in *calls_out -- [0] whole calls, [1] the
 * region take, [2] env-step launches, [3] the fork to the exchange stream, [4] ncclAllGather, [5]
 * consume launches, [6] closing events and count copy (n_out >= 7).  Recorded only when
 * CF2_XCHG_HOST_TIMING=1 was set at cf2_xchg_create; reset != 0 clears them. */
int  cf2_xchg_host_times(cf2_xchg* x, double* ns_out, uint32_t n_out, uint64_t* calls_out, int reset);

/* Measurement support (no reference counterpart): streaming kernels over `bytes` (a multiple of
 * 16, both pointers 16-B aligned) with non-temporal accesses.  mode 0: copy src -> dst; mode 1:
 * read src only (bytes >= 4096; dst must hold 4 KB and is normally left untouched).  bench.py times
 * them on 2 GiB to measure the box's HBM rates. */
int  cf2_hbm_probe(void* dst_dev, const void* src_dev, size_t bytes, int mode, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CF2SIM_H */
