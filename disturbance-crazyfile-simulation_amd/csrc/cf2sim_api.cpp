// cf2sim_api.cpp -- C ABI (include/cf2sim.h) over the HIP kernels.
//
// The context owns the SoA state in HBM; every I/O buffer is a caller-owned device pointer.
// No entry point allocates, frees or synchronises after cf2_create, so cf2_step /
// cf2_reset can be captured into a hipGraph by the caller.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>
#include <new>

#include "../../include/cf2sim.h"
#include "cf2sim_internal.h"

using namespace cf2;

struct cf2_ctx {
    cf2_config cfg;
    KParams P;
    KTables T;
    KTables* tab_dev = nullptr;
    float* sf = nullptr;           // internal AoSoA state, state_bytes(N)
    uint8_t* hj_bits = nullptr;    // per-node HJ sign bits of the bound tables
    size_t hj_bits_bytes = 0;
    int device = 0;
};

static thread_local int g_last_hip_error = 0;

int cf2::hip_fail(hipError_t e) {
    g_last_hip_error = (int)e;
    return e == hipErrorOutOfMemory ? CF2_ERR_OUT_OF_MEMORY : CF2_ERR_HIP;
}

static int validate(const cf2_config* c) {
    if (!c) return CF2_ERR_INVALID_ARG;
    if (c->num_envs == 0 || c->num_envs > CF2_MAX_ENVS_PER_CTX) return CF2_ERR_INVALID_ARG;
    if (c->physics != CF2_PHYS_BULLET && c->physics != CF2_PHYS_SIMPLE) return CF2_ERR_INVALID_ARG;
    if (c->task != CF2_TASK_HOVER && c->task != CF2_TASK_HOVER_FREE) return CF2_ERR_INVALID_ARG;
    if (c->disturbance < CF2_DSTB_NONE || c->disturbance > CF2_DSTB_HJ) return CF2_ERR_INVALID_ARG;
    if (c->level_mode != CF2_LEVEL_FIXED && c->level_mode != CF2_LEVEL_BOLTZMANN) return CF2_ERR_INVALID_ARG;
    if (c->aggregate_phy_steps < 1 || c->aggregate_phy_steps > 4) return CF2_ERR_UNSUPPORTED;
    if (c->obs_rate < 1) return CF2_ERR_INVALID_ARG;
    if (c->buf_size < 1 || c->buf_size > 4) return CF2_ERR_UNSUPPORTED;
    if (c->use_ground_effect && c->physics != CF2_PHYS_BULLET) return CF2_ERR_UNSUPPORTED;
    if (c->num_levels < 1 || c->num_levels > CF2_NUM_LEVELS_MAX) return CF2_ERR_INVALID_ARG;
    if (c->time_step <= 0.0 || c->mass <= 0.0) return CF2_ERR_INVALID_ARG;
    const int M = c->num_drones > 0 ? c->num_drones : 1;
    if (M != 1 && M != 2 && M != 4 && M != 8) return CF2_ERR_UNSUPPORTED;
    if (c->num_envs % (uint32_t)M || c->env_id_offset % (uint32_t)M) return CF2_ERR_INVALID_ARG;
    if (M > 1 && c->physics != CF2_PHYS_BULLET) return CF2_ERR_UNSUPPORTED;
    return CF2_OK;
}

// Bytes one env-step of this configuration moves (state read + written once, the action, every
// step() output); per-episode writes excluded.  The same count as bench.py's
// algorithmic_bytes_per_env_step over the whole step() boundary (762 B for the bench workload).
static uint64_t step_bytes_per_env(const cf2_config* c) {
    const bool noise = c->observation_noise_on, dr = c->domain_randomization_on;
    const int ol = noise ? 13 : 17, B = c->buf_size;
    const bool held = (c->aggregate_phy_steps % c->obs_rate) != 0;
    const bool gust_or_const = c->disturbance == CF2_DSTB_CONST || c->disturbance == CF2_DSTB_GUST;
    const bool level = c->disturbance == CF2_DSTB_CONST || c->disturbance == CF2_DSTB_HJ ||
                       c->level_mode == CF2_LEVEL_BOLTZMANN;
    int persist = 13 + 8 + 4 * B + (noise ? 6 : 0) + (noise && held ? 10 : 0) + ol + 8;
    if (c->physics == CF2_PHYS_SIMPLE) persist += 3;
    if (c->use_motor_dynamics) persist += 4;
    const int rd_f = persist + (dr ? 15 : 0) + (gust_or_const ? 3 : 0) + (level ? 1 : 0);
    const int wr_f = persist + (c->disturbance == CF2_DSTB_GUST ? 3 : 0);
    const int rd_i = 3 + (level ? 1 : 0) + (c->disturbance == CF2_DSTB_GUST ? 1 : 0);
    const int wr_i = 3 + (c->disturbance == CF2_DSTB_GUST ? 1 : 0);
    uint64_t b = 4u * (uint64_t)(rd_f + wr_f + rd_i + wr_i) + 16u;
    if (c->disturbance == CF2_DSTB_EXTERNAL) b += 12u;
    const int od = 2 * (ol + 4);
    return b + 4u * (uint64_t)od + 4u + 1u + 1u + 4u + 4u;
}
// Working-set bytes above which the step kernel's state stores are non-temporal: the Infinity
// Cache is 256 MB; measured on the bench workload, 327 680 envs (250 MB) run faster with plain
// stores and 393 216 envs (300 MB) with nt stores (profiles/r03_ab_nt_threshold.txt)
static const uint64_t NT_STATE_BYTES = 240ull << 20;

static void fill_tables(const cf2_config* c, KTables& T) {
    memset(&T, 0, sizeof(T));
    for (int k = 0; k < CF2_NUM_LEVELS_MAX; ++k) {
        T.level_values[k] = (float)c->level_values[k];
        T.level_cdf[k] = c->level_cdf[k];
        T.table_of_level[k] = -1;
    }
    for (int d = 0; d < 6; ++d)
        for (int k = 0; k < HJ_PTS; ++k) T.hj_grid[d][k] = c->hj_grid_points[d][k];
}

static void fill_params(const cf2_config* c, KParams& P) {
    memset(&P, 0, sizeof(P));
    P.N = c->num_envs;
    P.gid_off = c->env_id_offset;
    P.key0 = (uint32_t)(c->seed & 0xffffffffu);
    P.key1 = (uint32_t)(c->seed >> 32);
    P.agg = c->aggregate_phy_steps;
    P.obs_rate = c->obs_rate;
    P.buf_size = c->buf_size;
    P.use_latency = c->use_latency;
    P.use_motor_dyn = c->use_motor_dynamics;
    P.max_steps = c->max_episode_steps;
    P.auto_reset = c->auto_reset;
    P.reset_dist = c->enable_reset_distribution;
    P.dstb_mode = c->disturbance;
    P.level_mode = c->level_mode;
    P.num_levels = c->num_levels;
    P.gust_dur = c->gust_duration;
    P.noise = c->observation_noise_on;
    P.dr = c->domain_randomization_on;
    P.phys = c->physics;
    P.held_persistent = (c->aggregate_phy_steps % c->obs_rate) != 0;
    P.need_level = c->disturbance == CF2_DSTB_HJ || c->disturbance == CF2_DSTB_CONST ||
                   c->level_mode == CF2_LEVEL_BOLTZMANN;
    P.time_step = (float)c->time_step;
    P.mass = (float)c->mass;
    P.ixx = (float)c->ixx; P.iyy = (float)c->iyy; P.izz = (float)c->izz;
    P.ft0 = (float)c->ft0; P.ft1 = (float)c->ft1;
    P.K = (float)c->K; P.A = (float)c->A; P.B = (float)c->B;
    P.hover_x = (float)c->hover_x; P.hover_action = (float)c->hover_action;
    P.ou_sigma = (float)(0.2 * c->motor_thrust_noise);          // agents.py:206
    P.drag_xy = (float)c->drag_xy; P.drag_z = (float)c->drag_z;
    P.g_world = (float)c->gravity_world; P.g_agent = (float)c->gravity_agent;
    P.arm = (float)c->arm;
    P.prop_xy = (float)c->prop_xy; P.prop_z = (float)c->prop_z;
    P.prop_mass = (float)c->prop_mass; P.prop_inertia = (float)c->prop_inertia;
    P.prop_speed_gain = (float)c->prop_speed_gain;
    P.lin_damping = (float)c->lin_damping; P.ang_damping = (float)c->ang_damping;
    P.vmax = (float)c->max_coord_velocity;
    for (int k = 0; k < 3; ++k) P.init_xyz[k] = (float)c->init_xyz[k];
    P.pos_lim = (float)c->reset_pos_lim; P.angle_lim = (float)c->reset_angle_lim; P.yaw_lim = (float)c->reset_yaw_lim;
    P.vel_lim = (float)c->reset_vel_lim; P.rate_lim = (float)c->reset_rate_lim;
    P.yaw_rate_lim = (float)c->reset_yaw_rate_lim;
    P.action_std = (float)c->action_init_std; P.motor_std = (float)c->motor_init_std;
    const double f = c->domain_randomization;
    const double dr_val[9] = {c->time_step, c->mass, c->ixx, c->iyy, c->izz, c->ft0, c->ft1,
                              c->motor_time_constant, c->thrust2weight};
    for (int k = 0; k < 9; ++k) {                                  // base.py:253-259 bounds
        P.dr_lo[k] = (float)(dr_val[k] - f * dr_val[k]);
        P.dr_hi[k] = (float)(dr_val[k] + f * dr_val[k]);
    }
    P.pos_std = (float)c->pos_norm_std; P.pos_unif = (float)c->pos_unif_range;
    P.vel_std = (float)c->vel_norm_std;
    P.rot_std = (float)c->rot_norm_std; P.rot_unif = (float)c->rot_unif_range;
    {                                                              // sensors.py:123-127
        const double dt = 1.0 / c->sim_freq;
        const double sgd = c->gyro_noise_density / sqrt(dt);
        const double sbgd = sqrt(-(sgd * sgd) * (c->gyro_bias_corr_time / 2.0) *
                                 (exp(-2.0 * dt / c->gyro_bias_corr_time) - 1.0));
        P.pgd = (float)exp(-dt / c->gyro_bias_corr_time);
        P.sbgd = (float)sbgd;
    }
    P.gyro_rw = (float)c->gyro_random_walk; P.gyro_ton = (float)c->gyro_turn_on_bias_sigma;
    P.lpf_gain = (float)c->lpf_gain; P.lpf_ratio = (float)c->lpf_ratio;
    P.pen_action = (float)c->penalty_action; P.pen_angle = (float)c->penalty_angle;
    P.pen_spin = (float)c->penalty_spin; P.pen_term = (float)c->penalty_terminal;
    P.pen_vel = (float)c->penalty_velocity; P.pen_z = (float)c->penalty_z;
    P.pen_arp = (float)c->penalty_arp; P.pen_dist = (float)c->penalty_dist;
    for (int k = 0; k < 3; ++k) {
        P.target_pos[k] = (float)c->target_pos[k];
        P.target_rpy[k] = (float)c->target_rpy[k];
        P.target_rate[k] = (float)c->target_rate[k];
    }
    P.done_rp = (float)c->done_rp_limit; P.done_rate_deg = (float)c->done_rate_limit_deg;
    P.done_zmin = (float)c->done_z_min;
    P.cost_xy = (float)c->cost_xy_lim; P.cost_z = (float)c->cost_z_lim; P.cost_rp = (float)c->cost_rp_lim;
    P.cost_vel = (float)c->cost_vel_lim; P.cost_rate = (float)c->cost_rate_lim;
    P.level_fixed = (float)c->dstb_level;
    for (int k = 0; k < 3; ++k) {
        P.umax[k] = (float)c->dstb_umax[k];
        P.umax_d[k] = c->dstb_umax[k];
        P.uni_hi[k] = c->dstb_uniform_hi[k];
    }
    P.num_drones = c->num_drones > 0 ? c->num_drones : 1;
    P.downwash_on = c->downwash_on;
    for (int k = 0; k < 3; ++k) P.dw_coeff[k] = (float)c->dw_coeff[k];
    P.prop_radius = (float)c->prop_radius;
    P.formation_dx = (float)c->formation_dx;
    P.formation_dz = (float)c->formation_dz;
    P.ground_effect = c->use_ground_effect ? 1 : 0;
    P.gnd_eff_coeff = (float)c->gnd_eff_coeff;
    P.gnd_eff_h_clip = (float)c->gnd_eff_h_clip;
    P.gust_p = (float)c->gust_onset_prob;
    P.gust_max = (float)c->gust_max_level;
    P.tab = nullptr;
    P.V = nullptr;
    P.hj_bits = nullptr;
    P.nt_state = (uint64_t)c->num_envs * step_bytes_per_env(c) > NT_STATE_BYTES ? 1u : 0u;
}

extern "C" {

int cf2_abi_version(void) { return CF2SIM_ABI_VERSION; }
size_t cf2_config_sizeof(void) { return sizeof(cf2_config); }
int cf2_last_hip_error(void) { return g_last_hip_error; }

const char* cf2_status_string(int s) {
    switch (s) {
    case CF2_OK: return "ok";
    case CF2_ERR_INVALID_ARG: return "invalid argument";
    case CF2_ERR_OUT_OF_MEMORY: return "out of device memory";
    case CF2_ERR_HIP: return "HIP runtime error";
    case CF2_ERR_UNSUPPORTED: return "unsupported configuration";
    case CF2_ERR_NO_TABLE: return "HJ disturbance requested but no value table bound";
    default: return "unknown status";
    }
}

int cf2_create(const cf2_config* cfg, cf2_ctx** out_ctx) {
    if (!out_ctx) return CF2_ERR_INVALID_ARG;
    *out_ctx = nullptr;
    const int v = validate(cfg);
    if (v) return v;
    cf2_ctx* ctx = new (std::nothrow) cf2_ctx();
    if (!ctx) return CF2_ERR_OUT_OF_MEMORY;
    ctx->cfg = *cfg;
    fill_params(cfg, ctx->P);
    fill_tables(cfg, ctx->T);
    {   // the reset-only parameters the kernels read from the device tables
        KTables& T = ctx->T;
        const KParams& P = ctx->P;
        for (int k = 0; k < 3; ++k) T.init_xyz[k] = P.init_xyz[k];
        T.pos_lim = P.pos_lim; T.angle_lim = P.angle_lim; T.yaw_lim = P.yaw_lim;
        T.vel_lim = P.vel_lim; T.rate_lim = P.rate_lim; T.yaw_rate_lim = P.yaw_rate_lim;
        T.action_std = P.action_std; T.motor_std = P.motor_std;
        T.hover_x = P.hover_x; T.hover_action = P.hover_action;
        for (int k = 0; k < 9; ++k) { T.dr_lo[k] = P.dr_lo[k]; T.dr_hi[k] = P.dr_hi[k]; }
    }
    hipError_t e = hipGetDevice(&ctx->device);
    if (e == hipSuccess) e = query_occupancy(ctx->P);      // this device, this config's kernel instances
    if (e != hipSuccess) { delete ctx; return hip_fail(e); }
    const size_t N = cfg->num_envs;
    e = hipMalloc((void**)&ctx->tab_dev, sizeof(KTables));
    if (e == hipSuccess) e = hipMemcpy(ctx->tab_dev, &ctx->T, sizeof(KTables), hipMemcpyHostToDevice);
    ctx->P.tab = ctx->tab_dev;
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->sf, state_bytes((uint32_t)N));
    if (e == hipSuccess) e = launch_init(ctx->P, ctx->sf, 0);
    if (e == hipSuccess) e = hipStreamSynchronize(0);
    if (e != hipSuccess) {
        (void)hipFree(ctx->sf);
        (void)hipFree(ctx->tab_dev);
        delete ctx;
        return hip_fail(e);
    }
    *out_ctx = ctx;
    return CF2_OK;
}

int cf2_destroy(cf2_ctx* ctx) {
    if (!ctx) return CF2_ERR_INVALID_ARG;
    hipError_t e1 = hipFree(ctx->sf);
    (void)hipFree(ctx->tab_dev);
    if (ctx->hj_bits) (void)hipFree(ctx->hj_bits);
    delete ctx;
    if (e1 != hipSuccess) return hip_fail(e1);
    return CF2_OK;
}

int cf2_device_errors(cf2_ctx* ctx, uint32_t* flags_out, int clear) {
    if (!ctx || !flags_out) return CF2_ERR_INVALID_ARG;
    // synchronous: waits for the kernels issued so far (all streams of the device)
    hipError_t e = hipDeviceSynchronize();
    uint32_t* dev = &ctx->tab_dev->dev_err;
    if (e == hipSuccess) e = hipMemcpy(flags_out, dev, sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && clear && *flags_out) e = hipMemset(dev, 0, sizeof(uint32_t));
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_layout_get(const cf2_ctx* ctx, cf2_layout* o) {
    if (!ctx || !o) return CF2_ERR_INVALID_ARG;
    memset(o, 0, sizeof(*o));
    o->num_envs = ctx->cfg.num_envs;
    o->num_float_fields = NF;
    o->num_int_fields = NI;
    o->obs_len = ctx->cfg.observation_noise_on ? 13 : 17;
    o->obs_dim = 2 * (o->obs_len + 4);
    o->f_pos = F_POS; o->f_quat = F_QUAT; o->f_vel = F_VEL; o->f_omega = F_OMEGA; o->f_rpy = F_RPY;
    o->f_motor = F_MOTOR; o->f_ou = F_OU; o->f_abuf = F_ABUF; o->f_bias = F_BIAS; o->f_lpf = F_LPF;
    o->f_held = F_HELD; o->f_obs_prev = F_OBS_PREV; o->f_hist_act = F_HIST_ACT; o->f_param = F_PARAM;
    o->f_dstb = F_DSTB;
    o->i_ep_step = I_EP_STEP; o->i_rng = I_RNG; o->i_flags = I_FLAGS; o->i_level = I_LEVEL; o->i_gust = I_GUST;
    o->num_params = NUM_PARAMS;
    o->f_motor_lo = F_MOTOR_LO;
    return CF2_OK;
}

int cf2_bind_hj_tables(cf2_ctx* ctx, const float* V_dev, int num_tables, const int32_t* table_of_level) {
    if (!ctx || !V_dev || num_tables <= 0 || !table_of_level) return CF2_ERR_INVALID_ARG;
    for (int l = 0; l < ctx->cfg.num_levels; ++l)
        if (table_of_level[l] < -1 || table_of_level[l] >= num_tables) return CF2_ERR_INVALID_ARG;
    // the sign-table kernel indexes nodes in 32 bits
    if ((uint64_t)num_tables * (uint64_t)HJ_TABLE > (uint64_t)UINT32_MAX) return CF2_ERR_INVALID_ARG;
    // V may have been written on any stream of the caller (torch side streams do not synchronise
    // with the null stream), and step kernels still in flight may read the current tables and
    // bits: a binding is a setup-time call, so it waits for all device work first
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail(e);
    // Derived per-node sign bits (distur_gener's rule over the 7 taps around each node): the
    // env-step gathers one byte per env instead of 7 floats.  Derived once per binding: rebind
    // after changing the table contents.  Derived into a new buffer when the old one is too
    // small; nothing of the context changes until the derivation succeeded.
    const size_t need = (size_t)num_tables * (size_t)HJ_TABLE;
    uint8_t* bits = ctx->hj_bits;
    const bool fresh = need > ctx->hj_bits_bytes;
    if (fresh) {
        e = hipMalloc(&bits, need);
        if (e != hipSuccess) return hip_fail(e);
    }
    e = launch_hj_sign_table(V_dev, (uint32_t)num_tables, bits, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    KTables T = ctx->T;
    for (int l = 0; l < ctx->cfg.num_levels; ++l) T.table_of_level[l] = table_of_level[l];
    // only the level -> table map: a whole-block upload would also clear the device error word, and
    // with it any flag the kernels recorded before the rebind (cf2_device_errors reports them)
    if (e == hipSuccess)
        e = hipMemcpy(ctx->tab_dev->table_of_level, T.table_of_level, sizeof(T.table_of_level), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (fresh) (void)hipFree(bits);
        else {   // the old buffer was partly overwritten: the context has no valid tables now
            ctx->P.V = nullptr;
            ctx->P.hj_bits = nullptr;
        }
        return hip_fail(e);
    }
    if (fresh) {
        if (ctx->hj_bits) (void)hipFree(ctx->hj_bits);
        ctx->hj_bits = bits;
        ctx->hj_bits_bytes = need;
    }
    ctx->T = T;
    ctx->P.V = V_dev;
    ctx->P.hj_bits = ctx->hj_bits;
    return CF2_OK;
}

int cf2_reset(cf2_ctx* ctx, const uint8_t* mask_dev, float* obs_dev, void* stream) {
    if (!ctx) return CF2_ERR_INVALID_ARG;
    const hipError_t e = launch_reset(ctx->P, ctx->sf, mask_dev, obs_dev, (hipStream_t)stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_step(cf2_ctx* ctx, const float* act_dev, const float* dstb_dev, float* obs_dev, float* rew_dev,
             uint8_t* done_dev, uint8_t* trunc_dev, float* cost_dev, float* level_dev, float* final_obs_dev,
             void* stream) {
    if (!ctx || !act_dev || !obs_dev || !rew_dev || !done_dev) return CF2_ERR_INVALID_ARG;
    if (ctx->cfg.disturbance == CF2_DSTB_EXTERNAL && !dstb_dev) return CF2_ERR_INVALID_ARG;
    if (ctx->cfg.disturbance == CF2_DSTB_HJ && !ctx->P.V) return CF2_ERR_NO_TABLE;
    if (ctx->P.ground_effect) return CF2_ERR_UNSUPPORTED;       // physics plug-in only (cf2sim.h)
    if (((uintptr_t)act_dev & 15u) != 0 || ((uintptr_t)obs_dev & 15u) != 0) return CF2_ERR_INVALID_ARG;
    if (final_obs_dev && ((uintptr_t)final_obs_dev & 7u) != 0) return CF2_ERR_INVALID_ARG;
    StepIO io{ctx->sf, act_dev, dstb_dev, obs_dev, rew_dev, done_dev, trunc_dev, cost_dev, level_dev,
              final_obs_dev};
    const hipError_t e = launch_step(ctx->P, io, (hipStream_t)stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_step_packed(cf2_ctx* ctx, const float* act_dev, float* obs_dev, float* rew_dev, uint8_t* done_dev,
                    uint8_t* trunc_dev, float* cost_dev, float* level_dev, uint32_t* packed_dev, uint32_t* scratch_dev,
                    uint32_t cap, void* stream) {
    if (!ctx || !act_dev || !obs_dev || !rew_dev || !done_dev || !packed_dev || !scratch_dev) return CF2_ERR_INVALID_ARG;
    if (cap > ctx->P.N) return CF2_ERR_INVALID_ARG;
    if (ctx->cfg.disturbance == CF2_DSTB_EXTERNAL) return CF2_ERR_INVALID_ARG;
    if (ctx->cfg.disturbance == CF2_DSTB_HJ && !ctx->P.V) return CF2_ERR_NO_TABLE;
    if (ctx->P.ground_effect) return CF2_ERR_UNSUPPORTED;
    if (((uintptr_t)act_dev & 15u) != 0 || ((uintptr_t)obs_dev & 15u) != 0 || ((uintptr_t)packed_dev & 15u) != 0 ||
        ((uintptr_t)scratch_dev & 3u) != 0)
        return CF2_ERR_INVALID_ARG;
    StepIO io{ctx->sf, act_dev, nullptr, obs_dev, rew_dev, done_dev, trunc_dev, cost_dev, level_dev, nullptr};
    const PackIO pio{packed_dev, scratch_dev, cap};
    const hipError_t e = launch_step_packed(ctx->P, io, pio, (hipStream_t)stream);
    if (e == hipErrorNotSupported) return CF2_ERR_UNSUPPORTED;
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_collect_step(cf2_ctx* ctx, const float* act_dev, float* obs_dev, float* rew_dev, uint8_t* done_dev,
                     uint8_t* trunc_dev, float* final_obs_dev, const float* packed_dev, uint32_t obs_dim, int precision,
                     uint64_t seed, uint32_t counter, uint32_t row_offset, float* act_out_dev, float* val_out_dev,
                     float* logp_out_dev, void* stream) {
    if (!ctx || !act_dev || !obs_dev || !rew_dev || !done_dev || !packed_dev || !act_out_dev || !val_out_dev ||
        !logp_out_dev)
        return CF2_ERR_INVALID_ARG;
    if (act_out_dev == act_dev) return CF2_ERR_INVALID_ARG;
    if (ctx->cfg.disturbance == CF2_DSTB_EXTERNAL || ctx->P.ground_effect) return CF2_ERR_UNSUPPORTED;
    if (ctx->cfg.disturbance == CF2_DSTB_HJ && !ctx->P.V) return CF2_ERR_NO_TABLE;
    if (((uintptr_t)act_dev & 15u) != 0 || ((uintptr_t)obs_dev & 15u) != 0 || ((uintptr_t)act_out_dev & 15u) != 0 ||
        ((uintptr_t)packed_dev & 15u) != 0)
        return CF2_ERR_INVALID_ARG;
    if (final_obs_dev && ((uintptr_t)final_obs_dev & 7u) != 0) return CF2_ERR_INVALID_ARG;
    const uint32_t od = ctx->P.noise ? 34u : 42u;
    if (obs_dim != od) return CF2_ERR_INVALID_ARG;
    if (precision != CF2_POLICY_BF16X3 || od != 34u) return CF2_ERR_UNSUPPORTED;
    StepIO io{ctx->sf, act_dev, nullptr, obs_dev, rew_dev, done_dev, trunc_dev, nullptr, nullptr, final_obs_dev};
    PolicyIO pio{packed_dev, (uint32_t)seed, (uint32_t)(seed >> 32), counter, row_offset, act_out_dev, val_out_dev,
                 logp_out_dev};
    const hipError_t e = launch_collect(ctx->P, io, pio, (hipStream_t)stream);
    if (e == hipErrorNotSupported) return CF2_ERR_UNSUPPORTED;
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_collect_rollout(cf2_ctx* ctx, int K, float* act_dev, float* obs_dev, float* rew_dev, uint8_t* done_dev,
                        uint8_t* trunc_dev, float* final_obs_dev, const float* packed_dev, uint32_t obs_dim,
                        int precision, uint64_t seed, uint32_t counter, uint32_t row_offset, float* val_dev,
                        float* logp_dev, void* stream) {
    if (!ctx || K < 1 || !act_dev || !obs_dev || !rew_dev || !done_dev || !packed_dev || !val_dev || !logp_dev)
        return CF2_ERR_INVALID_ARG;
    if (ctx->cfg.disturbance == CF2_DSTB_EXTERNAL || ctx->P.ground_effect) return CF2_ERR_UNSUPPORTED;
    if (ctx->cfg.disturbance == CF2_DSTB_HJ && !ctx->P.V) return CF2_ERR_NO_TABLE;
    if (((uintptr_t)act_dev & 15u) != 0 || ((uintptr_t)obs_dev & 7u) != 0 || ((uintptr_t)packed_dev & 15u) != 0)
        return CF2_ERR_INVALID_ARG;
    if (final_obs_dev && ((uintptr_t)final_obs_dev & 7u) != 0) return CF2_ERR_INVALID_ARG;
    const uint32_t od = ctx->P.noise ? 34u : 42u;
    if (obs_dim != od) return CF2_ERR_INVALID_ARG;
    if (precision != CF2_POLICY_BF16X3 || od != 34u) return CF2_ERR_UNSUPPORTED;
    StepIO io{ctx->sf, act_dev, nullptr, obs_dev, rew_dev, done_dev, trunc_dev, nullptr, nullptr, final_obs_dev};
    PolicyIO pio{packed_dev, (uint32_t)seed, (uint32_t)(seed >> 32), counter, row_offset, act_dev, val_dev, logp_dev};
    const hipError_t e = launch_collect_rollout(ctx->P, io, pio, (uint32_t)K, (hipStream_t)stream);
    if (e == hipErrorNotSupported) return CF2_ERR_UNSUPPORTED;
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_physics_step(cf2_ctx* ctx, const float* act_dev, const float* dstb_dev, float time_step, void* stream) {
    if (!ctx || !act_dev || ((uintptr_t)act_dev & 15u) != 0) return CF2_ERR_INVALID_ARG;
    if (!(time_step < 1.0f)) return CF2_ERR_INVALID_ARG;       // NaN or absurd step
    const hipError_t e = launch_physics(ctx->P, ctx->sf, act_dev, dstb_dev, time_step, (hipStream_t)stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_set_ground_effect(cf2_ctx* ctx, int on) {
    if (!ctx) return CF2_ERR_INVALID_ARG;
    if (on && ctx->cfg.physics != CF2_PHYS_BULLET) return CF2_ERR_UNSUPPORTED;   // SimplePhysics has none
    ctx->P.ground_effect = on ? 1 : 0;
    ctx->cfg.use_ground_effect = on ? 1 : 0;
    return CF2_OK;
}

int cf2_rollout(cf2_ctx* ctx, int K, const float* act_dev, size_t act_stride_elems, float* obs_dev, float* rew_dev,
                uint8_t* done_dev, uint8_t* trunc_dev, float* cost_dev, float* level_dev, float* final_obs_dev,
                void* stream) {
    if (!ctx || K < 1 || !act_dev || !obs_dev || !rew_dev || !done_dev) return CF2_ERR_INVALID_ARG;
    const size_t n = ctx->cfg.num_envs;
    if (K > 1 && act_stride_elems < n * 4) return CF2_ERR_INVALID_ARG;
    if (act_stride_elems > (size_t)UINT32_MAX) return CF2_ERR_INVALID_ARG;   // the kernel strides in 32 bits
    if ((act_stride_elems & 3u) != 0 || ((uintptr_t)act_dev & 15u) != 0) return CF2_ERR_INVALID_ARG;
    if (((uintptr_t)obs_dev & 7u) != 0 || (final_obs_dev && ((uintptr_t)final_obs_dev & 7u) != 0))
        return CF2_ERR_INVALID_ARG;
    if (ctx->cfg.disturbance == CF2_DSTB_EXTERNAL) return CF2_ERR_UNSUPPORTED;   // one dstb tensor per step
    if (ctx->P.ground_effect) return CF2_ERR_UNSUPPORTED;       // physics plug-in only (cf2sim.h)
    if (ctx->cfg.disturbance == CF2_DSTB_HJ && !ctx->P.V) return CF2_ERR_NO_TABLE;
    StepIO io{ctx->sf, act_dev, nullptr, obs_dev, rew_dev, done_dev, trunc_dev, cost_dev, level_dev, final_obs_dev};
    const hipError_t e = launch_rollout(ctx->P, io, (uint32_t)K, (uint32_t)act_stride_elems, (hipStream_t)stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_get_state(const cf2_ctx* ctx, float* state_f_dev, int32_t* state_i_dev, void* stream) {
    if (!ctx || !state_f_dev || !state_i_dev) return CF2_ERR_INVALID_ARG;
    const hipError_t e = launch_state_convert(ctx->P, ctx->sf, state_f_dev, state_i_dev, 1, (hipStream_t)stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}
int cf2_set_state(cf2_ctx* ctx, const float* state_f_dev, const int32_t* state_i_dev, void* stream) {
    if (!ctx || !state_f_dev || !state_i_dev) return CF2_ERR_INVALID_ARG;
    const hipError_t e = launch_state_convert(ctx->P, ctx->sf, const_cast<float*>(state_f_dev),
                                              const_cast<int32_t*>(state_i_dev), 0, (hipStream_t)stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

int cf2_hj_disturbance(const cf2_config* cfg, const float* V_dev, const float* states_dev, uint32_t n, float level,
                       float* dstb_dev, float* uopt_dev, void* stream) {
    if (!cfg || !V_dev || !states_dev || !dstb_dev) return CF2_ERR_INVALID_ARG;
    if (!(level <= 3.0f)) return CF2_ERR_INVALID_ARG;            // assert disturbance <= 3.0 (distur_gener.py:154)
    // the grid nodes travel by value in the kernel arguments: no device table, no allocation, no
    // host synchronisation (the call can be captured into a hipGraph)
    HjGrid G;
    for (int d = 0; d < 6; ++d)
        for (int k = 0; k < HJ_PTS; ++k) G.p[d][k] = cfg->hj_grid_points[d][k];
    double umax[3];
    for (int k = 0; k < 3; ++k) umax[k] = cfg->dstb_umax[k];
    const hipError_t e = launch_hj(G, umax, V_dev, states_dev, n, level, dstb_dev, uopt_dev, (hipStream_t)stream);
    return e == hipSuccess ? CF2_OK : hip_fail(e);
}

}  // extern "C"
