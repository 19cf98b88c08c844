/*
 * cf2_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline.  The product path (libcf2sim.so) never
 * links or calls it.
 *
 * Scalar AoS C, one env at a time, compiled twice: REAL=double (the restatement proper)
 * and REAL=float (same op order in fp32, used to separate fp32 rounding from logic bugs).
 * Every function cites the reference code it restates (paths relative to
 * /root/reference/phoenix_drone_simulation/).
 *
 * Parity status (see DESIGN.md section "Oracle"):
 *   - agents.py / control.py / physics.py force+torque assembly, utils.py, sensors.py,
 *     base.py history/reset order, hover*.py reward/done/info, distur_gener.py and
 *     GridProcessing.py: pinned against golden vectors produced by running the reference's
 *     own Python (tests/golden/make_golden.py).
 *   - bc.stepSimulation() (bullet3 3.21 btMultiBody, third-party, not in the reference):
 *     restated from the published algorithm; parity vs PyBullet UNPINNED (pybullet absent).
 *   - RNG: the reference draws from numpy's global MT19937; this restatement and the HIP
 *     kernel share a counter-based Philox4x32-10 stream instead, so noise-on runs match the
 *     reference statistically, and match the HIP kernel draw-for-draw.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../include/cf2sim.h"

#ifndef REAL
#define REAL double
#endif
#define R(x) ((REAL)(x))

/* libm of the REAL type: R_SQRT is the square root (not a reciprocal square root), RSIN sin, ... */
#if defined(ORACLE_F32)
#define R_SQRT sqrtf
#define RSIN sinf
#define RCOS cosf
#define RLOG logf
#define RATAN2 atan2f
#define RASIN asinf
#define RFABS fabsf
#define REXP expf
#else
#define R_SQRT sqrt
#define RSIN sin
#define RCOS cos
#define RLOG log
#define RATAN2 atan2
#define RASIN asin
#define RFABS fabs
#define REXP exp
#endif

/* ------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11 "Parallel random numbers: as easy as 1, 2, 3").   */
/* ------------------------------------------------------------------------------------ */
void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

enum { TAG_STEP = 1, TAG_RESET = 2, TAG_PHYS = 3 };

typedef struct { uint32_t key[2]; uint32_t gid, ctr, tag; } rng_t;

static void rng_block(const rng_t* g, uint32_t block, uint32_t out[4]) {
    uint32_t c[4] = {block, g->ctr, g->gid, g->tag};
    orc_philox4x32_10(c, g->key, out);
}
/* 24-bit uniform in [0,1): identical value in fp32 and fp64 */
static REAL u01(uint32_t x) { return (REAL)(x >> 8) * R(5.9604644775390625e-08); }
/* Box-Muller pair from two u32: z0 = r cos, z1 = r sin */
static void box_muller(uint32_t a, uint32_t b, REAL* z0, REAL* z1) {
    REAL u1 = ((REAL)(a >> 8) + R(1.0)) * R(5.9604644775390625e-08); /* (0,1] */
    REAL u2 = (REAL)(b >> 8) * R(5.9604644775390625e-08);
    REAL r = R_SQRT(R(-2.0) * RLOG(u1));
    REAL th = R(6.283185307179586) * u2;
    *z0 = r * RCOS(th);
    *z1 = r * RSIN(th);
}
/* n normals from consecutive blocks starting at block b0 (pairs use u32 (2k,2k+1)) */
static void rng_normals(const rng_t* g, uint32_t b0, int n, REAL* z) {
    uint32_t buf[4];
    for (int k = 0; k < n; k += 2) {
        int w = k;              /* u32 index of this pair */
        if ((w & 3) == 0) rng_block(g, b0 + (uint32_t)(w >> 2), buf);
        REAL z0, z1;
        box_muller(buf[w & 3], buf[(w & 3) + 1], &z0, &z1);
        z[k] = z0;
        if (k + 1 < n) z[k + 1] = z1;
    }
}

/* ------------------------------------------------------------------------------------ */
/* Rotation helpers (PyBullet C-API semantics; bullet3 btMatrix3x3 / pybullet.c)         */
/* ------------------------------------------------------------------------------------ */
/* pybullet getMatrixFromQuaternion: btMatrix3x3(q), row-major, s = 2/|q|^2 */
void orc_rotmat(const REAL q[4], REAL Rm[9]) {
    REAL x = q[0], y = q[1], z = q[2], w = q[3];
    REAL d = x * x + y * y + z * z + w * w;
    REAL s = R(2.0) / d;
    REAL xs = x * s, ys = y * s, zs = z * s;
    REAL wx = w * xs, wy = w * ys, wz = w * zs;
    REAL xx = x * xs, xy = x * ys, xz = x * zs;
    REAL yy = y * ys, yz = y * zs, zz = z * zs;
    Rm[0] = R(1.0) - (yy + zz); Rm[1] = xy - wz;               Rm[2] = xz + wy;
    Rm[3] = xy + wz;               Rm[4] = R(1.0) - (xx + zz); Rm[5] = yz - wx;
    Rm[6] = xz - wy;               Rm[7] = yz + wx;               Rm[8] = R(1.0) - (xx + yy);
}
/* pybullet getQuaternionFromEuler (normalised), same formula as envs/utils.py:58-82 */
void orc_quat_from_euler(const REAL rpy[3], REAL q[4]) {
    REAL phi = rpy[0] * R(0.5), the = rpy[1] * R(0.5), psi = rpy[2] * R(0.5);
    REAL sp = RSIN(phi), cp = RCOS(phi), st = RSIN(the), ct = RCOS(the), ss = RSIN(psi), cs = RCOS(psi);
    REAL x = sp * ct * cs - cp * st * ss;
    REAL y = cp * st * cs + sp * ct * ss;
    REAL z = cp * ct * ss - sp * st * cs;
    REAL w = cp * ct * cs + sp * st * ss;
    REAL len = R_SQRT(x * x + y * y + z * z + w * w);
    q[0] = x / len; q[1] = y / len; q[2] = z / len; q[3] = w / len;
}
/* pybullet getEulerFromQuaternion (agents.py:446 readback) */
void orc_euler_from_quat(const REAL q[4], REAL rpy[3]) {
    REAL sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
    REAL sarg = R(-2.0) * (q[0] * q[2] - q[3] * q[1]);
    if (sarg <= R(-0.99999)) {
        rpy[0] = R(0.0); rpy[1] = R(-0.5) * R(3.141592653589793); rpy[2] = R(2.0) * RATAN2(q[0], -q[1]);
    } else if (sarg >= R(0.99999)) {
        rpy[0] = R(0.0); rpy[1] = R(0.5) * R(3.141592653589793); rpy[2] = R(2.0) * RATAN2(-q[0], q[1]);
    } else {
        rpy[0] = RATAN2(R(2.0) * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz);
        rpy[1] = RASIN(sarg);
        rpy[2] = RATAN2(R(2.0) * (q[0] * q[1] + q[3] * q[2]), squ + sqx - sqy - sqz);
    }
}
/* distur_gener.quat2euler  adversarial_generation/FasTrack_data/distur_gener.py:186-207 */
void orc_quat2euler(const REAL q[4], REAL e[3]) {
    REAL x = q[0], y = q[1], z = q[2], w = q[3];
    REAL t0 = R(2.0) * (w * x + y * z);
    REAL t1 = R(1.0) - R(2.0) * (x * x + y * y);
    e[0] = RATAN2(t0, t1);
    REAL t2 = R(2.0) * (w * y - z * x);
    t2 = t2 > R(1.0) ? R(1.0) : t2;
    t2 = t2 < R(-1.0) ? R(-1.0) : t2;
    e[1] = RASIN(t2);
    REAL t3 = R(2.0) * (w * z + x * y);
    REAL t4 = R(1.0) - R(2.0) * (y * y + z * z);
    e[2] = RATAN2(t3, t4);
}
static void matvec(const REAL M[9], const REAL v[3], REAL o[3]) {
    o[0] = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
    o[1] = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
    o[2] = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
}
static void matTvec(const REAL M[9], const REAL v[3], REAL o[3]) {
    o[0] = M[0] * v[0] + M[3] * v[1] + M[6] * v[2];
    o[1] = M[1] * v[0] + M[4] * v[1] + M[7] * v[2];
    o[2] = M[2] * v[0] + M[5] * v[1] + M[8] * v[2];
}
static REAL norm3(const REAL v[3]) { return R_SQRT(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
static REAL clampr(REAL x, REAL lo, REAL hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* ------------------------------------------------------------------------------------ */
/* HJ disturbance: distur_gener.py:19-183 with Grid.get_index GridProcessing.py:52-71     */
/* ------------------------------------------------------------------------------------ */
static int grid_nearest(const double* pts, int n, double s) {
    /* np.searchsorted(side='left'): first i with pts[i] >= s */
    int idx = 0;
    while (idx < n && pts[idx] < s) ++idx;
    if (idx > 0 && (idx == n || fabs(s - pts[idx - 1]) < fabs(s - pts[idx]))) return idx - 1;
    return idx;
}
static float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }
/* states: [roll, pitch, yaw, p, q, r]; returns dOpt, uOpt (opt_dstb_non_hcl / opt_ctrl_non_hcl) */
void orc_hj_eval(const cf2_config* cfg, const float* V, const double states[6], double level,
                 double dopt[3], double uopt[3], int32_t idx_out[6]) {
    int idx[6];
    for (int d = 0; d < 6; ++d) idx[d] = grid_nearest(cfg->hj_grid_points[d], CF2_HJ_PTS, states[d]);
    long stride[6];
    stride[5] = 1;
    for (int d = 4; d >= 0; --d) stride[d] = stride[d + 1] * CF2_HJ_PTS;
    long c = 0;
    for (int d = 0; d < 6; ++d) c += idx[d] * stride[d];
    if (idx_out) for (int d = 0; d < 6; ++d) idx_out[d] = idx[d];
    for (int i = 0; i < 3; ++i) {
        int d = 3 + i;                      /* only dims 3,4,5 enter opt_dstb (distur_gener.py:111-116) */
        float Vc = V[c];
        float L, Rr;                        /* numerators of left/right one-sided differences (float32) */
        if (idx[d] == 0) {                  /* non-periodic lower boundary, distur_gener.py:73-82 */
            float Vn = V[c + stride[d]];
            float lb = Vc + fabsf(Vn - Vc) * sgnf(Vc);
            L = Vc - lb; Rr = Vn - Vc;
        } else if (idx[d] == CF2_HJ_PTS - 1) {  /* upper boundary, :83-92 */
            float Vp = V[c - stride[d]];
            float rb = Vc + fabsf(Vc - Vp) * sgnf(Vc);
            L = Vc - Vp; Rr = rb - Vc;
        } else {
            float Vp = V[c - stride[d]], Vn = V[c + stride[d]];
            L = Vc - Vp; Rr = Vn - Vc;
        }
        /* (L/dx + R/dx)/2 > 0  <=>  L + R > 0 exactly (float32 operands, float64 quotients) */
        int pos = L > -Rr;
        double um = cfg->dstb_umax[i];
        double dm = level * um;             /* dmax = disturbance * umax, :160 */
        dopt[i] = pos ? -dm : dm;
        uopt[i] = pos ? -um : um;
    }
}

/* ------------------------------------------------------------------------------------ */
/* Env state (AoS mirror of the reference's attributes)                                   */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    /* bullet base state: p, q (x,y,z,w) world orientation, v world, w world */
    REAL p[3], q[4], v[3], ww[3];
    /* CrazyFlieAgent attributes */
    REAL rpy[3], wb[3];                 /* drone.rpy, drone.rpy_dot (body) */
    REAL x[4], ou[4], abuf[4][4];
    REAL xl[4];                         /* f32 build: low word of the motor state (x + xl) */
    int aidx;
    REAL last_action[4];
    int last_action_is_view;            /* drone.last_action aliases action_buffer[-1] */
    int props_on;                       /* a physics sub-step ran since the reset (prop joints spin) */
    /* per-env params (DR) */
    REAL dt, m, J[3], k0, k1, A[4], B[4], K[4];
    /* sensor */
    REAL bias[3], lpf[3], held[10];
    /* history */
    REAL obs_prev[17];
    REAL hact[2][4];
    int halias[2];                      /* action_history entry aliases action_buffer[-1] */
    int ep_step, iteration;
    uint32_t rng_ctr;
    /* disturbance */
    REAL dstb[3];
    REAL level;
    int level_idx;
    int gust_left;
} orc_env;

typedef struct {
    cf2_config cfg;
    int n;
    orc_env* e;
    const float* V;           /* HJ tables [num_tables][15^6] */
    int num_tables;
    int32_t table_of_level[CF2_NUM_LEVELS_MAX];
    int threads;              /* OpenMP threads of orc_step (formations are independent) */
} orc_ctx;

static int obs_len(const cf2_config* c) { return c->observation_noise_on ? 13 : 17; }

static rng_t mk_rng(const orc_ctx* X, int i, uint32_t tag) {
    rng_t g;
    g.key[0] = (uint32_t)(X->cfg.seed & 0xffffffffu);
    g.key[1] = (uint32_t)(X->cfg.seed >> 32);
    g.gid = X->cfg.env_id_offset + (uint32_t)i;
    g.ctr = X->e[i].rng_ctr;
    g.tag = tag;
    return g;
}

/* CrazyFlieAgent.apply_action agents.py:259-298 (+ PWM.act control.py:94-100,
 * OUNoise.noise utils.py:130-134).  Returns forces f[4] and yaw torque. */
static void apply_action(const orc_ctx* X, orc_env* E, const REAL a[4], const REAL ou_n[4],
                         REAL f[4], REAL* tz) {
    const cf2_config* c = &X->cfg;
    REAL pwm[4];
    for (int j = 0; j < 4; ++j) E->last_action[j] = a[j];
    E->last_action_is_view = 0;
    if (c->use_latency) {
        REAL delayed[4];
        for (int j = 0; j < 4; ++j) delayed[j] = E->abuf[E->aidx][j];
        for (int j = 0; j < 4; ++j) E->abuf[E->aidx][j] = a[j];
        E->aidx = (E->aidx + 1) % c->buf_size;
        for (int j = 0; j < 4; ++j) pwm[j] = R(30000.0) + clampr(delayed[j], R(-1.0), R(1.0)) * R(30000.0);
    } else {
        for (int j = 0; j < 4; ++j) pwm[j] = R(30000.0) + clampr(a[j], R(-1.0), R(1.0)) * R(30000.0);
    }
    REAL sigma = R(0.2 * c->motor_thrust_noise);
    for (int j = 0; j < 4; ++j) {       /* dx = theta*(mu - x) + sigma*randn; x += dx */
        REAL xo = E->ou[j];
        REAL dx = R(0.15) * (R(0.0) - xo) + sigma * ou_n[j];
        E->ou[j] = xo + dx;
    }
    for (int j = 0; j < 4; ++j) {
        REAL tn = pwm[j] / R(60000.0);
        REAL noisy;
        if (c->use_motor_dynamics) {
            REAL rot = R_SQRT(tn);
#if defined(ORACLE_F32) && !defined(ORACLE_REF_MOTOR)
            /* the HIP kernel's form: x += B (rot - x) with x kept as an unevaluated pair x + xl
             * (TwoSum), so the 5 ms recurrence does not accumulate fp32 rounding.  Equal to
             * A x + B rot for A = 1 - B (agents.py:288); see DESIGN.md section 5.  The fp64 build
             * and the f32ref build (ORACLE_REF_MOTOR: fp32 in the reference's own form) keep
             * A x + B rot literally. */
            {
                REAL inc = E->B[j] * ((rot - E->x[j]) - E->xl[j]);
                REAL sum = E->x[j] + inc, bb = sum - E->x[j];                       /* TwoSum */
                REAL lo = ((E->x[j] - (sum - bb)) + (inc - bb)) + E->xl[j];
                E->x[j] = sum + lo;                                                  /* renormalise */
                E->xl[j] = lo - (E->x[j] - sum);
            }
#else
            E->x[j] = E->A[j] * E->x[j] + E->B[j] * rot;
#endif
            noisy = (R(1.0) + E->ou[j]) * (E->x[j] * E->x[j]);
        } else {
            noisy = (R(1.0) + E->ou[j]) * tn;
        }
        REAL nn = clampr(noisy, R(0.0), R(1.0));
        f[j] = E->K[j] * nn;
    }
    REAL t[4];
    for (int j = 0; j < 4; ++j) t[j] = E->k1 * f[j] + E->k0;
    *tz = (-t[0] + t[1] - t[2] + t[3]);
}

/* update_information agents.py:434-453 (bullet readback) */
static void update_information(orc_env* E) {
    REAL Rm[9];
    orc_euler_from_quat(E->q, E->rpy);
    orc_rotmat(E->q, Rm);
    matTvec(Rm, E->ww, E->wb);
}

/* One physics sub-step, CF2_PHYS_BULLET: PybulletPhysicsWithAdversary.step_forward
 * physics.py:213-250 (force/torque assembly, drag) followed by a restatement of bullet3 3.21
 * btMultiBodyDynamicsWorld::stepSimulation for the cf21x_bullet.urdf multibody:
 *   applyGravity; computeAccelerationsArticulatedBodyAlgorithmMultiDof (base spatial
 *   velocity in the base frame, external wrench, damping k1=k2=0.04 times the base mass /
 *   inertia, gyroscopic w x Iw, Coriolis w x v bias) ; applyDeltaVeeMultiDof with the
 *   +-m_maxCoordinateVelocity clamp; prop velocity motors (target x*100 rad/s, always within
 *   the 0.01 N m * dt impulse bound) reached exactly; stepPositionsMultiDof (base position
 *   Euler, exp-map quaternion update with the pi/4 clamp and Taylor branch, normalise).
 * The 4 prop links (1e-9 kg, 1e-9 kg m^2) are kept as a gyrostat: composite inertia, rotor
 * momentum h = Ip * sum(axis_i * qdot_i) z_b, its change across the motor constraint and the
 * prop links' own angular damping.  The zero-mass centre-of-mass link passes its wrench
 * straight to the base (invD = 0 guard in the ABA). */
static void bullet_substep(const orc_ctx* X, orc_env* E, const REAL a[4], const REAL dstb[3],
                           const REAL ou_n[4], int first_after_reset, REAL dw) {
    const cf2_config* c = &X->cfg;
    REAL xprev[4];
    for (int j = 0; j < 4; ++j) xprev[j] = E->x[j];
    REAL f[4], tz;
    apply_action(X, E, a, ou_n, f, &tz);

    REAL Rm[9];
    orc_rotmat(E->q, Rm);
    /* drag: rpm = x^2*25000; drag = R . (-DRAG * sum(2 pi rpm/60) * v) ; applied in LINK_FRAME of
     * link 4 => world force R . drag (physics.py:232-241, agents.py:300-309) */
    REAL ssum = R(0.0);
    for (int j = 0; j < 4; ++j) {
        REAL rpm = E->x[j] * E->x[j] * R(25000.0);
        ssum += R(2.0) * R(3.141592653589793) * rpm / R(60.0);
    }
    REAL dcoef[3] = {R(-1.0) * R(c->drag_xy) * ssum, R(-1.0) * R(c->drag_xy) * ssum, R(-1.0) * R(c->drag_z) * ssum};
    REAL dl[3] = {dcoef[0] * E->v[0], dcoef[1] * E->v[1], dcoef[2] * E->v[2]};
    REAL drag1[3], dragw[3];
    matvec(Rm, dl, drag1);
    matvec(Rm, drag1, dragw);

    /* body-frame external torque: props at (+-L, +-L, Lz) with force f z_b (agents.py:311-321,
     * cf21x_bullet.urdf prop1..4_joint), yaw torque and adversary torques on link 4 in its frame
     * (agents.py:330-337, 517-533).  Only dstb[0], dstb[1] are applied (physics.py:228-229). */
    REAL L = R(c->prop_xy);
    /* ground effect (BasePhysics.calculate_ground_effect physics.py:27-58, applied with the prop
     * forces physics.py:243-246 while |roll|, |pitch| < pi/2 of the last readback): prop heights
     * z_i = (p + R o_i)_z (getLinkStates), clipped at GND_EFF_H_CLIP (agents.py:156) */
    if (c->use_ground_effect && fabs((double)E->rpy[0]) < 1.5707963267948966 && fabs((double)E->rpy[1]) < 1.5707963267948966) {
        const REAL ox[4] = {L, -L, -L, L}, oy[4] = {-L, -L, L, L}, oz = R(c->prop_z);
        for (int j = 0; j < 4; ++j) {
            REAL z = E->p[2] + (Rm[6] * ox[j] + Rm[7] * oy[j] + Rm[8] * oz);
            if (z < R(c->gnd_eff_h_clip)) z = R(c->gnd_eff_h_clip);
            const REAL rr = R(c->prop_radius) / (R(4.0) * z);
            f[j] = f[j] + f[j] * R(c->gnd_eff_coeff) * (rr * rr);
        }
    }
    REAL tb[3];
    tb[0] = L * (-f[0] - f[1] + f[2] + f[3]) + dstb[0];
    tb[1] = L * (-f[0] + f[1] + f[2] - f[3]) + dstb[1];
    tb[2] = tz;
    REAL fsum = f[0] + f[1] + f[2] + f[3];

    REAL mp = R(c->prop_mass), Ip = R(c->prop_inertia), Lz = R(c->prop_z);
    REAL mtot = E->m + R(4.0) * mp;
    REAL g = R(c->gravity_world);
    /* world force; dw = downwash from formation mates (multi-drone extension), a force along -z
     * of the body applied at the centre of mass (LINK_FRAME, posObj 0) */
    REAL Fw[3];
    REAL fz = fsum - dw;
    Fw[0] = Rm[2] * fz + dragw[0];
    Fw[1] = Rm[5] * fz + dragw[1];
    Fw[2] = Rm[8] * fz + dragw[2] - g * mtot;

    /* base spatial velocity in the base frame */
    REAL wb[3], vb[3];
    matTvec(Rm, E->ww, wb);
    matTvec(Rm, E->v, vb);
    REAL wn = norm3(wb), vn = norm3(vb);
    REAL ld = R(c->lin_damping), ad = R(c->ang_damping);
    /* composite inertia (props locked about x/y; spin dof handled as rotor momentum) */
    REAL Ic[3];
    Ic[0] = E->J[0] + R(4.0) * Ip + R(4.0) * mp * (L * L + Lz * Lz);
    Ic[1] = E->J[1] + R(4.0) * Ip + R(4.0) * mp * (L * L + Lz * Lz);
    Ic[2] = E->J[2] + R(4.0) * Ip + R(4.0) * mp * (L * L + L * L);
    /* rotor spin (relative joint rates qdot_i = x_i*100, axes -z,+z,-z,+z) */
    REAL kq = R(c->prop_speed_gain);
    REAL sp_old = first_after_reset ? R(0.0) : kq * (-xprev[0] + xprev[1] - xprev[2] + xprev[3]);
    REAL sp_new = kq * (-E->x[0] + E->x[1] - E->x[2] + E->x[3]);
    REAL h_old = Ip * sp_old;
    /* angular: Ic wdot = tau - w x (Ic w + h z) - damping(base) - damping(props) - dh/dt */
    REAL Iw[3] = {Ic[0] * wb[0], Ic[1] * wb[1], Ic[2] * wb[2] + h_old};
    REAL gyro[3] = {wb[1] * Iw[2] - wb[2] * Iw[1], wb[2] * Iw[0] - wb[0] * Iw[2], wb[0] * Iw[1] - wb[1] * Iw[0]};
    REAL dampa = ad * (R(1.0) + wn);
    REAL tdamp[3] = {E->J[0] * wb[0] * dampa, E->J[1] * wb[1] * dampa, E->J[2] * wb[2] * dampa};
    /* prop link angular damping: each prop spins at w_b + a_i qdot_i z */
    REAL pd[3] = {R(0.0), R(0.0), R(0.0)};
    {
        const REAL ax[4] = {R(-1.0), R(1.0), R(-1.0), R(1.0)};
        for (int j = 0; j < 4; ++j) {
            REAL qd = first_after_reset ? R(0.0) : kq * xprev[j];
            REAL wp[3] = {wb[0], wb[1], wb[2] + ax[j] * qd};
            REAL k = Ip * ad * (R(1.0) + norm3(wp));
            pd[0] += k * wp[0]; pd[1] += k * wp[1]; pd[2] += k * wp[2];
        }
    }
    REAL dt = E->dt;
    REAL wdot_b[3];
    wdot_b[0] = (tb[0] - gyro[0] - tdamp[0] - pd[0]) / Ic[0];
    wdot_b[1] = (tb[1] - gyro[1] - tdamp[1] - pd[1]) / Ic[1];
    wdot_b[2] = (tb[2] - gyro[2] - tdamp[2] - pd[2] - Ip * (sp_new - sp_old) / dt) / Ic[2];
    /* linear: vdot_w = F_w/m - R (0.04 (1+|v|) v_b) * m_base/m  (w x v bias cancels) */
    REAL dampl = ld * (R(1.0) + vn) * E->m / mtot;
    REAL vdot_w[3], wdot_w[3];
    for (int k = 0; k < 3; ++k) vdot_w[k] = Fw[k] / mtot - dampl * E->v[k];
    matvec(Rm, wdot_b, wdot_w);
    REAL vmax = R(c->max_coord_velocity);
    for (int k = 0; k < 3; ++k) {
        E->ww[k] = clampr(E->ww[k] + wdot_w[k] * dt, -vmax, vmax);
        E->v[k] = clampr(E->v[k] + vdot_w[k] * dt, -vmax, vmax);
    }
    /* stepPositionsMultiDof */
    for (int k = 0; k < 3; ++k) E->p[k] += dt * E->v[k];
    {
        REAL ang = norm3(E->ww);
        if (ang * dt > R(0.7853981633974483)) ang = R(0.7853981633974483) / dt;
        REAL axs[3];
        if (ang < R(0.001)) {
            REAL s = R(0.5) * dt - (dt * dt * dt) * R(0.020833333333) * ang * ang;
            for (int k = 0; k < 3; ++k) axs[k] = E->ww[k] * s;
        } else {
            REAL s = RSIN(R(0.5) * ang * dt) / ang;
            for (int k = 0; k < 3; ++k) axs[k] = E->ww[k] * s;
        }
        REAL cw = RCOS(R(0.5) * ang * dt);
        /* q_new = (axs, cw) (x) q */
        REAL qx = E->q[0], qy = E->q[1], qz = E->q[2], qw = E->q[3];
        REAL nx = cw * qx + axs[0] * qw + axs[1] * qz - axs[2] * qy;
        REAL ny = cw * qy + axs[1] * qw + axs[2] * qx - axs[0] * qz;
        REAL nz = cw * qz + axs[2] * qw + axs[0] * qy - axs[1] * qx;
        REAL nw = cw * qw - axs[0] * qx - axs[1] * qy - axs[2] * qz;
        REAL len = R_SQRT(nx * nx + ny * ny + nz * nz + nw * nw);
        E->q[0] = nx / len; E->q[1] = ny / len; E->q[2] = nz / len; E->q[3] = nw / len;
    }
    update_information(E);
}

/* SimplePhysics.step_forward physics.py:130-200 */
static void simple_substep(const orc_ctx* X, orc_env* E, const REAL a[4], const REAL ou_n[4]) {
    const cf2_config* c = &X->cfg;
    REAL f[4], tz;
    apply_action(X, E, a, ou_n, f, &tz);
    REAL Rm[9];
    orc_rotmat(E->q, Rm);
    REAL fsum = f[0] + f[1] + f[2] + f[3];
    REAL g = R(c->gravity_world);
    REAL Fw[3] = {Rm[2] * fsum - R(0.0) * E->m, Rm[5] * fsum - R(0.0) * E->m, Rm[8] * fsum - g * E->m};
    /* (..) * self.drone.L / np.sqrt(2), evaluated left to right */
    REAL tx = (-f[0] - f[1] + f[2] + f[3]) * R(c->arm) / R_SQRT(R(2.0));
    REAL ty = (-f[0] + f[1] + f[2] - f[3]) * R(c->arm) / R_SQRT(R(2.0));
    REAL* w = E->wb;
    REAL Jw[3] = {E->J[0] * w[0], E->J[1] * w[1], E->J[2] * w[2]};
    REAL cr[3] = {w[1] * Jw[2] - w[2] * Jw[1], w[2] * Jw[0] - w[0] * Jw[2], w[0] * Jw[1] - w[1] * Jw[0]};
    REAL t[3] = {tx - cr[0], ty - cr[1], tz - cr[2]};
    /* rpy_dot_dot = J_INV . torques with J_INV = np.linalg.inv(J) (multiplication by 1/J) */
    REAL wdd[3] = {(R(1.0) / E->J[0]) * t[0], (R(1.0) / E->J[1]) * t[1], (R(1.0) / E->J[2]) * t[2]};
    REAL acc[3] = {Fw[0] / E->m, Fw[1] / E->m, Fw[2] / E->m};
    REAL dt = E->dt;
    for (int k = 0; k < 3; ++k) E->v[k] += dt * acc[k];
    for (int k = 0; k < 3; ++k) E->wb[k] += dt * wdd[k];
    for (int k = 0; k < 3; ++k) E->p[k] += dt * E->v[k];
    for (int k = 0; k < 3; ++k) E->rpy[k] += dt * E->wb[k];
    orc_quat_from_euler(E->rpy, E->q);
    if (E->p[2] < R(0.0)) E->p[2] = R(0.0);
    /* keep the (unused) bullet angular velocity consistent: resetBaseVelocity(R^T wb) */
    matTvec(Rm, E->wb, E->ww);
}

/* SensorNoise.add_noise_to_omega sensors.py:121-134 ; n[9] = bias, random walk, turn-on */
static void omega_noise(const cf2_config* c, orc_env* E, const REAL w[3], const REAL* n, REAL out[3]) {
    double dt = 1.0 / c->sim_freq;
    double sgd = c->gyro_noise_density / sqrt(dt);
    double sbgd = sqrt(-(sgd * sgd) * (c->gyro_bias_corr_time / 2.0) * (exp(-2.0 * dt / c->gyro_bias_corr_time) - 1.0));
    double pgd = exp(-dt / c->gyro_bias_corr_time);
    for (int k = 0; k < 3; ++k) E->bias[k] = R(pgd) * E->bias[k] + R(sbgd) * n[k];
    for (int k = 0; k < 3; ++k)
        out[k] = w[k] + E->bias[k] + R(c->gyro_random_walk) * n[3 + k] + R(c->gyro_turn_on_bias_sigma) * n[6 + k];
}

/* compute_observation hover_free.py:168-200 (== hover.py:146-178).  rng block base for
 * this observation call; writes obs (13 with noise, 17 without). */
static void compute_observation(const orc_ctx* X, orc_env* E, const rng_t* g, uint32_t base, REAL* obs) {
    const cf2_config* c = &X->cfg;
    if (!c->observation_noise_on) {
        for (int k = 0; k < 3; ++k) obs[k] = E->p[k];
        for (int k = 0; k < 4; ++k) obs[3 + k] = E->q[k];
        for (int k = 0; k < 3; ++k) obs[7 + k] = E->v[k];
        for (int k = 0; k < 3; ++k) obs[10 + k] = E->wb[k];
        for (int k = 0; k < 4; ++k) obs[13 + k] = E->last_action[k];
        return;
    }
    REAL om[3];
    if (E->iteration % c->obs_rate == 0) {
        REAL n[18];
        uint32_t u[8];
        rng_normals(g, base, 18, n);
        rng_block(g, base + 4, u);    /* u32 16..19: u[0..3] ; base+5: u32 20..23 */
        rng_block(g, base + 5, u + 4);
        /* sensors.py:75-118 */
        REAL pos[3], vel[3], rot[3];
        for (int k = 0; k < 3; ++k) {
            REAL uu = u01(u[2 + k]);     /* u32 18,19,20 */
            REAL uo = R(-c->pos_unif_range) + (R(c->pos_unif_range) - R(-c->pos_unif_range)) * uu;
            pos[k] = E->p[k] + (R(c->pos_norm_std) * n[k] + uo);
        }
        for (int k = 0; k < 3; ++k) vel[k] = E->v[k] + R(c->vel_norm_std) * n[3 + k] + R(0.0);
        omega_noise(c, E, E->wb, n + 6, om);
        const REAL lo[3] = {R(-3.141592653589793), R(-1.5707963267948966), R(-3.141592653589793)};
        for (int k = 0; k < 3; ++k) {
            REAL uu = u01(u[5 + k]);     /* u32 21,22,23 */
            REAL uo = R(-c->rot_unif_range) + (R(c->rot_unif_range) - R(-c->rot_unif_range)) * uu;
            REAL th = R(c->rot_norm_std) * n[15 + k] + uo;
            rot[k] = clampr(E->rpy[k] + th, lo[k], -lo[k]);
        }
        REAL qn[4];
        orc_quat_from_euler(rot, qn);
        for (int k = 0; k < 3; ++k) E->held[k] = pos[k];
        for (int k = 0; k < 4; ++k) E->held[3 + k] = qn[k];
        for (int k = 0; k < 3; ++k) E->held[7 + k] = vel[k];
    } else {
        REAL n[10];
        rng_normals(g, base, 9, n);
        omega_noise(c, E, E->wb, n, om);
    }
    /* LowPassFilter.apply utils.py:102-105 */
    for (int k = 0; k < 3; ++k)
        E->lpf[k] = (R(1.0) - R(c->lpf_ratio)) * E->lpf[k] + R(c->lpf_gain) * R(c->lpf_ratio) * om[k];
    for (int k = 0; k < 10; ++k) obs[k] = E->held[k];
    for (int k = 0; k < 3; ++k) obs[10 + k] = E->lpf[k];
}

/* compute_done hover_free.py:449-461 / :124-136, hover.py:102-114 */
static int compute_done(const cf2_config* c, const orc_env* E) {
    int rp = RFABS(E->rpy[0]) > R(c->done_rp_limit) || RFABS(E->rpy[1]) > R(c->done_rp_limit);
    int rt = 0;
    for (int k = 0; k < 3; ++k) rt |= (R(180.0) * RFABS(E->wb[k]) / R(3.141592653589793)) > R(c->done_rate_limit_deg);
    int z = E->p[2] < R(c->done_z_min);
    return rp || rt || z;
}

/* compute_reward hover_free.py:206-235 / hover.py:184-202 (np.sum of the 6 penalties in order) */
static REAL compute_reward(const cf2_config* c, const orc_env* E, const REAL a[4], int done) {
    REAL na[4], ad[4];
    for (int k = 0; k < 4; ++k) { na[k] = R(0.5) * (clampr(a[k], R(-1.0), R(1.0)) + R(1.0)); ad[k] = a[k] - E->last_action[k]; }
    REAL nna = R_SQRT(na[0] * na[0] + na[1] * na[1] + na[2] * na[2] + na[3] * na[3]);
    REAL nad = R_SQRT(ad[0] * ad[0] + ad[1] * ad[1] + ad[2] * ad[2] + ad[3] * ad[3]);
    REAL dr[3], dw[3], dp[3];
    for (int k = 0; k < 3; ++k) {
        dr[k] = E->rpy[k] - R(c->target_rpy[k]);
        dw[k] = E->wb[k] - R(c->target_rate[k]);
        dp[k] = E->p[k] - R(c->target_pos[k]);
    }
    REAL p_action = R(c->penalty_action) * nna;
    REAL p_arp = R(c->penalty_arp) * nad;
    REAL p_rpy = R(c->penalty_angle) * norm3(dr);
    REAL p_spin = R(c->penalty_spin) * norm3(dw);
    REAL p_term = done ? R(c->penalty_terminal) : R(0.0);
    REAL p_vel = R(c->penalty_velocity) * norm3(E->v);
    REAL pen = R(0.0);
    pen += p_rpy; pen += p_arp; pen += p_spin; pen += p_vel; pen += p_action; pen += p_term;
    REAL zd = R(c->penalty_z) * RFABS(E->p[2] - R(c->target_pos[2]));
    REAL dist = R(c->penalty_dist) * norm3(dp);
    return -pen - zd - dist;
}

/* compute_info hover_free.py:138-166 (cost flag; note state[10:13] = body rates and
 * state[13:16] = last_action[0:3], as indexed by the reference) */
static REAL compute_cost(const cf2_config* c, const orc_env* E) {
    REAL cost = R(0.0);
    if (RFABS(E->p[0]) > R(c->cost_xy_lim) || RFABS(E->p[1]) > R(c->cost_xy_lim) || E->p[2] > R(c->cost_z_lim)) cost = R(1.0);
    if (RFABS(E->rpy[0]) > R(c->cost_rp_lim) || RFABS(E->rpy[1]) > R(c->cost_rp_lim)) cost = R(1.0);
    for (int k = 0; k < 3; ++k) if (RFABS(E->wb[k]) > R(c->cost_vel_lim)) cost = R(1.0);
    for (int k = 0; k < 3; ++k) if (RFABS(E->last_action[k]) > R(c->cost_rate_lim)) cost = R(1.0);
    return cost;
}

/* action_history entry value: an alias of action_buffer[-1] or a stored copy (base.py:455-460) */
static void hist_value(const cf2_config* c, const orc_env* E, int slot, REAL out[4]) {
    for (int k = 0; k < 4; ++k)
        out[k] = E->halias[slot] ? E->abuf[c->buf_size - 1][k] : E->hact[slot][k];
}

/* compute_history base.py:305-321; obs_next computed by the caller */
static void compute_history(const cf2_config* c, orc_env* E, const REAL* obs_next, REAL* out) {
    int ol = obs_len(c);
    REAL a0[4], a1[4];
    hist_value(c, E, 0, a0);
    hist_value(c, E, 1, a1);
    int o = 0;
    for (int k = 0; k < ol; ++k) out[o++] = E->obs_prev[k];
    for (int k = 0; k < 4; ++k) out[o++] = a0[k];
    for (int k = 0; k < ol; ++k) out[o++] = obs_next[k];
    for (int k = 0; k < 4; ++k) out[o++] = a1[k];
    for (int k = 0; k < ol; ++k) E->obs_prev[k] = obs_next[k];
    /* action_history.append(drone.last_action) */
    E->halias[0] = E->halias[1];
    for (int k = 0; k < 4; ++k) E->hact[0][k] = E->hact[1][k];
    E->halias[1] = E->last_action_is_view;
    for (int k = 0; k < 4; ++k) E->hact[1][k] = E->last_action[k];
}

/* Boltzmann() envs/utils.py:27-39 via numpy choice(): cdf.searchsorted(u, side='right') */
static int boltzmann_index(const cf2_config* c, REAL u) {
    int i = 0;
    while (i < c->num_levels - 1 && !((double)u < c->level_cdf[i])) ++i;
    return i;
}

static void set_level(const orc_ctx* X, orc_env* E, int idx) {
    E->level_idx = idx;
    E->level = R(X->cfg.level_values[idx]);
}

/* DroneBaseEnv.reset base.py:420-464 with task_specific_reset hover_free.py:237-289,
 * apply_domain_randomization base.py:241-298; writes obs (obs_dim) */
/* ---- multi-drone extension (no reference implementation) ---- */
/* formation slot of drone k of a group of M: columns of 2, formation_dx apart in x, the second
 * drone of a column formation_dz above the first */
static void formation_offset(const cf2_config* c, uint32_t k, REAL off[3]) {
    const int M = c->num_drones > 0 ? c->num_drones : 1;
    const int ncol = (M + 1) / 2;
    off[0] = ((REAL)(int)(k / 2) - (REAL)(ncol - 1) * R(0.5)) * R(c->formation_dx);
    off[1] = R(0.0);
    off[2] = (REAL)(int)(k % 2) * R(c->formation_dz);
    if (M == 1) off[0] = off[2] = R(0.0);
}
/* gym-pybullet-drones BaseAviary._downwash, summed over the group's drones above drone n */
REAL orc_downwash(const cf2_config* c, const REAL pn[3], const REAL (*pos)[3], int M, int self) {
    REAL F = R(0.0);
    for (int j = 0; j < M; ++j) {
        if (j == self) continue;
        const REAL dz = pos[j][2] - pn[2];
        const REAL dx = pos[j][0] - pn[0], dy = pos[j][1] - pn[1];
        const REAL dxy = R_SQRT(dx * dx + dy * dy);
        if (dz > R(0.0) && dxy < R(10.0)) {
            const REAL rr = R(c->prop_radius) / (R(4.0) * dz);
            const REAL alpha = R(c->dw_coeff[0]) * rr * rr;
            const REAL beta = R(c->dw_coeff[1]) * dz + R(c->dw_coeff[2]);
            const REAL q = dxy / beta;
            F += alpha * REXP(R(-0.5) * q * q);
        }
    }
    return F;
}

static void reset_env(orc_ctx* X, int i, REAL* obs) {
    const cf2_config* c = &X->cfg;
    orc_env* E = &X->e[i];
    rng_t g = mk_rng(X, i, TAG_RESET);
    uint32_t u[16];
    rng_block(&g, 0, u); rng_block(&g, 1, u + 4); rng_block(&g, 2, u + 8); rng_block(&g, 3, u + 12);
    /* stale drone.rpy_dot (previous episode) for the gyro LPF (base.py:444) */
    REAL stale_wb[3] = {E->wb[0], E->wb[1], E->wb[2]};

    E->iteration = 0;
    E->ep_step = 0;
    E->props_on = 0;
    /* drone.reset() agents.py:377-386 */
    for (int j = 0; j < 4; ++j) E->x[j] = E->xl[j] = R(0.0);
    E->aidx = 0;
    for (int r = 0; r < 4; ++r) for (int j = 0; j < 4; ++j) E->abuf[r][j] = R(0.0);
    /* task_specific_reset */
    REAL pos[3] = {R(c->init_xyz[0]), R(c->init_xyz[1]), R(c->init_xyz[2])};
    {
        REAL off[3];
        formation_offset(c, (c->env_id_offset + (uint32_t)i) % (uint32_t)(c->num_drones > 0 ? c->num_drones : 1), off);
        for (int k = 0; k < 3; ++k) pos[k] += off[k];
    }
    REAL quat[4] = {R(0.0), R(0.0), R(0.0), R(1.0)};
    REAL vel[3] = {R(0.0), R(0.0), R(0.0)}, rate[3] = {R(0.0), R(0.0), R(0.0)};
    if (c->enable_reset_distribution) {
        for (int k = 0; k < 3; ++k) pos[k] += R(-c->reset_pos_lim) + (R(c->reset_pos_lim) - R(-c->reset_pos_lim)) * u01(u[k]);
        REAL rpy[3];
        rpy[0] = R(-c->reset_angle_lim) + (R(c->reset_angle_lim) - R(-c->reset_angle_lim)) * u01(u[4]);
        rpy[1] = R(-c->reset_angle_lim) + (R(c->reset_angle_lim) - R(-c->reset_angle_lim)) * u01(u[5]);
        rpy[2] = R(-c->reset_yaw_lim) + (R(c->reset_yaw_lim) - R(-c->reset_yaw_lim)) * u01(u[3]);
        orc_quat_from_euler(rpy, quat);
        for (int k = 0; k < 3; ++k) vel[k] = vel[k] + (R(-c->reset_vel_lim) + (R(c->reset_vel_lim) - R(-c->reset_vel_lim)) * u01(u[8 + k]));
        rate[0] = rate[0] + (R(-c->reset_rate_lim) + (R(c->reset_rate_lim) - R(-c->reset_rate_lim)) * u01(u[11]));
        rate[1] = rate[1] + (R(-c->reset_rate_lim) + (R(c->reset_rate_lim) - R(-c->reset_rate_lim)) * u01(u[12]));
        rate[2] = R(-c->reset_yaw_rate_lim) + (R(c->reset_yaw_rate_lim) - R(-c->reset_yaw_rate_lim)) * u01(u[7]);
        REAL nx[4];
        rng_normals(&g, 4, 4, nx);
        for (int j = 0; j < 4; ++j) E->x[j] = R(c->hover_x) + R(c->motor_init_std) * nx[j];
        REAL nb[16];
        rng_normals(&g, 5, 16, nb);
        for (int r = 0; r < c->buf_size; ++r)
            for (int j = 0; j < 4; ++j)
                E->abuf[r][j] = clampr(R(c->hover_action) + R(c->action_init_std) * nb[4 * r + j], R(-1.0), R(1.0));
    }
    /* drone.last_action = action_buffer[-1, :] (a view) */
    for (int j = 0; j < 4; ++j) E->last_action[j] = E->abuf[c->buf_size - 1][j];
    E->last_action_is_view = 1;
    /* resetBasePositionAndOrientation / resetBaseVelocity(angularVelocity = R^T rate) */
    for (int k = 0; k < 3; ++k) { E->p[k] = pos[k]; E->v[k] = vel[k]; }
    for (int k = 0; k < 4; ++k) E->q[k] = quat[k];
    {
        REAL Rm[9];
        orc_rotmat(quat, Rm);
        matTvec(Rm, rate, E->ww);
    }
    /* apply_domain_randomization base.py:241-298 */
    E->dt = R(c->time_step); E->m = R(c->mass); E->J[0] = R(c->ixx); E->J[1] = R(c->iyy); E->J[2] = R(c->izz);
    E->k0 = R(c->ft0); E->k1 = R(c->ft1);
    for (int j = 0; j < 4; ++j) { E->A[j] = R(c->A); E->B[j] = R(c->B); E->K[j] = R(c->K); }
    if (c->domain_randomization_on) {
        uint32_t d[16];
        rng_block(&g, 9, d); rng_block(&g, 10, d + 4); rng_block(&g, 11, d + 8); rng_block(&g, 12, d + 12);
        double fct = c->domain_randomization;
#define DRAW(val, ui) (R((val) - fct * (val)) + (R((val) + fct * (val)) - R((val) - fct * (val))) * u01(d[ui]))
        E->dt = DRAW(c->time_step, 0);
        E->m = DRAW(c->mass, 1);
        E->J[0] = DRAW(c->ixx, 2); E->J[1] = DRAW(c->iyy, 3); E->J[2] = DRAW(c->izz, 4);
        E->k0 = DRAW(c->ft0, 5); E->k1 = DRAW(c->ft1, 6);
        if (c->use_motor_dynamics) {
            for (int j = 0; j < 4; ++j) {
                REAL mtc = DRAW(c->motor_time_constant, 7 + j);
                REAL t2w = DRAW(c->thrust2weight, 11 + j);
                REAL T = mtc < E->dt ? E->dt : mtc;
                E->A[j] = R(1.0) - E->dt / T;
                E->B[j] = E->dt / T;
                E->K[j] = R(0.028) * R(c->gravity_agent) * t2w / R(4.0);  /* agents.py:224 (0.028 sic) */
            }
        }
#undef DRAW
    }
    /* per-episode disturbance parameters */
    {
        uint32_t w[4];
        rng_block(&g, 13, w);
        if (c->disturbance == CF2_DSTB_CONST) {
            for (int k = 0; k < 3; ++k) E->dstb[k] = (R(-1.0) + R(2.0) * u01(w[k])) * R(c->dstb_umax[k]) * E->level;
        } else {
            for (int k = 0; k < 3; ++k) E->dstb[k] = R(0.0);
        }
        E->gust_left = 0;
    }
    /* gyro_lpf.set(drone.rpy_dot) -- the stale value (base.py:444) */
    for (int k = 0; k < 3; ++k) E->lpf[k] = stale_wb[k];
    /* update_information */
    if (c->physics == CF2_PHYS_BULLET) {
        update_information(E);
    } else {
        REAL Rm[9];
        orc_euler_from_quat(E->q, E->rpy);
        orc_rotmat(E->q, Rm);
        matTvec(Rm, E->ww, E->wb);
    }
    /* obs = compute_observation(); histories filled with it; compute_history() */
    REAL o0[17], o1[17];
    compute_observation(X, E, &g, 32, o0);
    for (int k = 0; k < obs_len(c); ++k) E->obs_prev[k] = o0[k];
    E->halias[0] = E->halias[1] = 1;
    for (int s = 0; s < 2; ++s) for (int k = 0; k < 4; ++k) E->hact[s][k] = E->last_action[k];
    compute_observation(X, E, &g, 40, o1);
    compute_history(c, E, o1, obs);
    /* Boltzmann level redraw at the end of reset (hover_free.py:536) */
    if (c->level_mode == CF2_LEVEL_BOLTZMANN) set_level(X, E, boltzmann_index(c, u01(u[13])));
    E->rng_ctr += 1;
}

/* ------------------------------------------------------------------------------------ */
/* Public (test-only) API                                                                */
/* ------------------------------------------------------------------------------------ */
void* orc_create(const cf2_config* cfg) {
    orc_ctx* X = (orc_ctx*)calloc(1, sizeof(orc_ctx));
    X->cfg = *cfg;
    X->n = (int)cfg->num_envs;
    X->e = (orc_env*)calloc((size_t)X->n, sizeof(orc_env));
    for (int i = 0; i < X->n; ++i) {
        orc_env* E = &X->e[i];
        E->p[2] = R(1.0);                    /* AgentBase default xyz (0,0,1) */
        E->q[3] = R(1.0);
        E->dt = R(cfg->time_step); E->m = R(cfg->mass);
        E->J[0] = R(cfg->ixx); E->J[1] = R(cfg->iyy); E->J[2] = R(cfg->izz);
        E->k0 = R(cfg->ft0); E->k1 = R(cfg->ft1);
        for (int j = 0; j < 4; ++j) { E->A[j] = R(cfg->A); E->B[j] = R(cfg->B); E->K[j] = R(cfg->K); }
        E->level_idx = 0;
        E->level = R(cfg->dstb_level);
        if (cfg->level_mode == CF2_LEVEL_BOLTZMANN) {
            /* construction-time Boltzmann() draw (hover_free.py:488), rng counter 0xFFFFFFFF */
            rng_t g = mk_rng(X, i, TAG_RESET);
            g.ctr = 0xFFFFFFFFu;
            uint32_t u[4];
            rng_block(&g, 0, u);
            set_level(X, E, boltzmann_index(cfg, u01(u[0])));
        }
    }
    for (int l = 0; l < CF2_NUM_LEVELS_MAX; ++l) X->table_of_level[l] = -1;
    return X;
}
/* OpenMP threads used by orc_step (default 1; the bench's all-core CPU baseline raises it). */
void orc_set_threads(void* h, int threads) { ((orc_ctx*)h)->threads = threads; }
void orc_set_ground_effect(void* h, int on) { ((orc_ctx*)h)->cfg.use_ground_effect = on ? 1 : 0; }

void orc_destroy(void* h) {
    orc_ctx* X = (orc_ctx*)h;
    free(X->e);
    free(X);
}
void orc_bind_tables(void* h, const float* V, int num_tables, const int32_t* table_of_level) {
    orc_ctx* X = (orc_ctx*)h;
    X->V = V;
    X->num_tables = num_tables;
    for (int l = 0; l < X->cfg.num_levels && l < CF2_NUM_LEVELS_MAX; ++l) X->table_of_level[l] = table_of_level[l];
}

void orc_reset(void* h, const uint8_t* mask, double* obs) {
    orc_ctx* X = (orc_ctx*)h;
    int od = 2 * (obs_len(&X->cfg) + 4);
    REAL o[42];
    for (int i = 0; i < X->n; ++i) {
        if (mask && !mask[i]) continue;
        reset_env(X, i, o);
        if (obs) for (int k = 0; k < od; ++k) obs[(size_t)i * od + k] = (double)o[k];
    }
}

static void disturbance_for_step(orc_ctx* X, int i, const rng_t* g, const double* dstb_ext, REAL d[3]) {
    const cf2_config* c = &X->cfg;
    orc_env* E = &X->e[i];
    d[0] = d[1] = d[2] = R(0.0);
    uint32_t u[4];
    switch (c->disturbance) {
    case CF2_DSTB_EXTERNAL:
        for (int k = 0; k < 3; ++k) d[k] = R(dstb_ext[(size_t)i * 3 + k]);
        break;
    case CF2_DSTB_UNIFORM:
        rng_block(g, 0, u);
        for (int k = 0; k < 3; ++k) {
            /* gym Box.sample(): uniform(low, high) cast to float32 */
            float v = (float)(-c->dstb_uniform_hi[k] + (c->dstb_uniform_hi[k] - -c->dstb_uniform_hi[k]) * (double)u01(u[k]));
            d[k] = R(v);
        }
        break;
    case CF2_DSTB_CONST:
        for (int k = 0; k < 3; ++k) d[k] = E->dstb[k];
        break;
    case CF2_DSTB_GUST:
        rng_block(g, 0, u);
        if (E->gust_left == 0 && u01(u[0]) < R(c->gust_onset_prob)) {
            E->gust_left = c->gust_duration;
            REAL mag = R(c->gust_max_level) * u01(u[1]);
            for (int k = 0; k < 3; ++k)
                E->dstb[k] = ((u[2] >> k) & 1u ? R(-1.0) : R(1.0)) * mag * R(c->dstb_umax[k]);
        }
        if (E->gust_left > 0) {
            for (int k = 0; k < 3; ++k) d[k] = E->dstb[k];
            E->gust_left -= 1;
        } else {
            for (int k = 0; k < 3; ++k) E->dstb[k] = R(0.0);
        }
        break;
    case CF2_DSTB_HJ: {
        int t = X->table_of_level[E->level_idx];
        if (c->level_mode == CF2_LEVEL_FIXED) t = X->table_of_level[0];
        if (t < 0 || !X->V) break;
        REAL e[3];
        orc_quat2euler(E->q, e);
        /* states = quat2euler(get_state()[3:7]) ++ get_state()[10:13]  (hover_free.py:418-424) */
        double st[6] = {(double)e[0], (double)e[1], (double)e[2], (double)E->wb[0], (double)E->wb[1], (double)E->wb[2]};
        double dopt[3], uopt[3];
        orc_hj_eval(c, X->V + (size_t)t * 11390625u, st, (double)E->level, dopt, uopt, NULL);
        for (int k = 0; k < 3; ++k) d[k] = R(dopt[k]);
        break;
    }
    default: break;
    }
}

/* One env-step for every env (see cf2_step in include/cf2sim.h). */
void orc_step(void* h, const float* act, const double* dstb_ext, double* obs, double* rew,
              uint8_t* done_out, uint8_t* trunc_out, double* cost_out, double* level_out, double* final_obs) {
    orc_ctx* X = (orc_ctx*)h;
    const cf2_config* c = &X->cfg;
    int ol = obs_len(c), od = 2 * (ol + 4);
    const int M = c->num_drones > 0 ? c->num_drones : 1;
    /* formations touch only their own envs: they split across threads with identical results */
#pragma omp parallel for schedule(static) num_threads(X->threads > 0 ? X->threads : 1) if (X->threads > 1)
    for (int g0 = 0; g0 < X->n; g0 += M) {
      /* the drones of one formation advance their sub-steps in lock step: the downwash of sub-step
       * s uses every mate's position before that sub-step (single drones: M = 1) */
      REAL a_g[8][4], d_g[8][3], level_g[8];
      rng_t g_g[8];
      for (int m = 0; m < M; ++m) {
        const int i = g0 + m;
        g_g[m] = mk_rng(X, i, TAG_STEP);
        for (int k = 0; k < 4; ++k) a_g[m][k] = R(act[(size_t)i * 4 + k]);
        level_g[m] = X->e[i].level;
        disturbance_for_step(X, i, &g_g[m], dstb_ext, d_g[m]);
      }
      for (int s = 0; s < c->aggregate_phy_steps; ++s) {
        REAL pos[8][3];
        for (int m = 0; m < M; ++m)
          for (int k = 0; k < 3; ++k) pos[m][k] = X->e[g0 + m].p[k];
        for (int m = 0; m < M; ++m) {
          orc_env* E = &X->e[g0 + m];
          const REAL dw = (M > 1 && c->downwash_on) ? orc_downwash(c, pos[m], (const REAL(*)[3])pos, M, m) : R(0.0);
          REAL ou_n[4];
          rng_normals(&g_g[m], 1 + (uint32_t)s, 4, ou_n);
          if (c->physics == CF2_PHYS_BULLET) bullet_substep(X, E, a_g[m], d_g[m], ou_n, E->ep_step == 0 && s == 0 && !E->props_on, dw);
          else simple_substep(X, E, a_g[m], ou_n);
          REAL dummy[17];
          compute_observation(X, E, &g_g[m], 8 + 8 * (uint32_t)s, dummy);
          E->iteration += 1;
        }
      }
      for (int m = 0; m < M; ++m) {
        const int i = g0 + m;
        orc_env* E = &X->e[i];
        rng_t g = g_g[m];
        REAL* a = a_g[m];
        const REAL level_used = level_g[m];
        REAL on[17], o[42];
        compute_observation(X, E, &g, 8 + 8 * (uint32_t)c->aggregate_phy_steps, on);
        compute_history(c, E, on, o);
        int term = compute_done(c, E);
        REAL r = compute_reward(c, E, a, term);
        REAL cost = compute_cost(c, E);
        E->ep_step += 1;
        int trunc = c->max_episode_steps > 0 && E->ep_step >= c->max_episode_steps && !term;
        int done = term || trunc;
        if (rew) rew[i] = (double)r;
        if (done_out) done_out[i] = (uint8_t)done;
        if (trunc_out) trunc_out[i] = (uint8_t)trunc;
        if (cost_out) cost_out[i] = (double)cost;
        if (level_out) level_out[i] = (double)level_used;
        if (done && c->auto_reset) {
            if (final_obs) for (int k = 0; k < od; ++k) final_obs[(size_t)i * od + k] = (double)o[k];
            reset_env(X, i, o);         /* uses this step's rng counter under TAG_RESET */
            E->rng_ctr -= 1;            /* reset_env advanced it; the step advances it once below */
        }
        E->rng_ctr += 1;
        if (obs) for (int k = 0; k < od; ++k) obs[(size_t)i * od + k] = (double)o[k];
      }
    }
}

/* One physics sub-step of every env: the physics plugin's step_forward on its own
 * (PyBulletPhysics physics.py:91-124, SimplePhysics :130-200, PybulletPhysicsWithAdversary
 * :213-250), i.e. apply_action + force/torque assembly + drag + rigid-body step + readback, with no
 * observation, reward or counters around it (cf2_physics_step).  OU normals: Philox block 0 of
 * (rng counter, TAG_PHYS); the counter advances once per call.  dt_override > 0 replaces the
 * per-env time step for this call (BasePhysics.set_parameters physics.py:60-68). */
void orc_physics_step(void* h, const float* act, const double* dstb, double dt_override) {
    orc_ctx* X = (orc_ctx*)h;
    const cf2_config* c = &X->cfg;
    for (int i = 0; i < X->n; ++i) {
        orc_env* E = &X->e[i];
        rng_t g = mk_rng(X, i, TAG_PHYS);
        REAL a[4], d[3] = {R(0.0), R(0.0), R(0.0)}, ou_n[4];
        for (int k = 0; k < 4; ++k) a[k] = R(act[(size_t)i * 4 + k]);
        if (dstb) for (int k = 0; k < 3; ++k) d[k] = R(dstb[(size_t)i * 3 + k]);
        const REAL dt_saved = E->dt;
        if (dt_override > 0.0) E->dt = R(dt_override);
        rng_normals(&g, 0, 4, ou_n);
        if (c->physics == CF2_PHYS_BULLET) {
            if (c->use_ground_effect) orc_euler_from_quat(E->q, E->rpy);     /* drone.rpy of the last readback */
            bullet_substep(X, E, a, d, ou_n, E->ep_step == 0 && !E->props_on, R(0.0));
        } else {
            simple_substep(X, E, a, ou_n);
        }
        E->dt = dt_saved;
        E->props_on = 1;
        E->rng_ctr += 1;
    }
}

/* SoA snapshot in the HIP kernel's layout (DESIGN.md "State layout"). */
#define NF 108
#define NI 5
void orc_get_state(void* h, double* sf, int32_t* si) {
    orc_ctx* X = (orc_ctx*)h;
    const cf2_config* c = &X->cfg;
    size_t N = (size_t)X->n;
    for (size_t i = 0; i < N; ++i) {
        orc_env* E = &X->e[i];
        double f[NF];
        memset(f, 0, sizeof(f));
        for (int k = 0; k < 3; ++k) f[0 + k] = E->p[k];
        for (int k = 0; k < 4; ++k) f[3 + k] = E->q[k];
        for (int k = 0; k < 3; ++k) f[7 + k] = E->v[k];
        for (int k = 0; k < 3; ++k) f[10 + k] = c->physics == CF2_PHYS_BULLET ? E->ww[k] : E->wb[k];
        for (int k = 0; k < 3; ++k) f[13 + k] = E->rpy[k];
        for (int k = 0; k < 4; ++k) f[16 + k] = E->x[k];
        for (int k = 0; k < 4; ++k) f[20 + k] = E->ou[k];
        for (int r = 0; r < 4; ++r) for (int k = 0; k < 4; ++k) f[24 + 4 * r + k] = E->abuf[r][k];
        for (int k = 0; k < 3; ++k) f[40 + k] = E->bias[k];
        for (int k = 0; k < 3; ++k) f[43 + k] = E->lpf[k];
        for (int k = 0; k < 10; ++k) f[46 + k] = E->held[k];
        for (int k = 0; k < 17; ++k) f[56 + k] = E->obs_prev[k];
        for (int s = 0; s < 2; ++s) for (int k = 0; k < 4; ++k) f[73 + 4 * s + k] = E->hact[s][k];
        f[81] = E->dt; f[82] = E->m; f[83] = E->J[0]; f[84] = E->J[1]; f[85] = E->J[2];
        f[86] = E->k0; f[87] = E->k1;
        for (int k = 0; k < 4; ++k) { f[88 + k] = E->A[k]; f[92 + k] = E->B[k]; f[96 + k] = E->K[k]; }
        for (int k = 0; k < 3; ++k) f[100 + k] = E->dstb[k];
        f[103] = E->level;
        for (int k = 0; k < 4; ++k) f[104 + k] = E->xl[k];
        for (int k = 0; k < NF; ++k) sf[(size_t)k * N + i] = f[k];
        si[0 * N + i] = E->ep_step;
        si[1 * N + i] = (int32_t)E->rng_ctr;
        si[2 * N + i] = (E->aidx & 15) | (E->halias[0] << 4) | (E->halias[1] << 5) | (E->last_action_is_view << 6) | (E->props_on << 7);
        si[3 * N + i] = E->level_idx;
        si[4 * N + i] = E->gust_left;
    }
}
void orc_set_state(void* h, const double* sf, const int32_t* si) {
    orc_ctx* X = (orc_ctx*)h;
    const cf2_config* c = &X->cfg;
    size_t N = (size_t)X->n;
    for (size_t i = 0; i < N; ++i) {
        orc_env* E = &X->e[i];
#define F(k) ((REAL)sf[(size_t)(k) * N + i])
        for (int k = 0; k < 3; ++k) E->p[k] = F(0 + k);
        for (int k = 0; k < 4; ++k) E->q[k] = F(3 + k);
        for (int k = 0; k < 3; ++k) E->v[k] = F(7 + k);
        for (int k = 0; k < 4; ++k) E->x[k] = F(16 + k);
        for (int k = 0; k < 4; ++k) E->ou[k] = F(20 + k);
        for (int r = 0; r < 4; ++r) for (int k = 0; k < 4; ++k) E->abuf[r][k] = F(24 + 4 * r + k);
        for (int k = 0; k < 3; ++k) E->bias[k] = F(40 + k);
        for (int k = 0; k < 3; ++k) E->lpf[k] = F(43 + k);
        for (int k = 0; k < 10; ++k) E->held[k] = F(46 + k);
        for (int k = 0; k < 17; ++k) E->obs_prev[k] = F(56 + k);
        for (int s = 0; s < 2; ++s) for (int k = 0; k < 4; ++k) E->hact[s][k] = F(73 + 4 * s + k);
        E->dt = F(81); E->m = F(82); E->J[0] = F(83); E->J[1] = F(84); E->J[2] = F(85);
        E->k0 = F(86); E->k1 = F(87);
        for (int k = 0; k < 4; ++k) { E->A[k] = F(88 + k); E->B[k] = F(92 + k); E->K[k] = F(96 + k); }
        for (int k = 0; k < 3; ++k) E->dstb[k] = F(100 + k);
        E->level = F(103);
        for (int k = 0; k < 4; ++k) E->xl[k] = F(104 + k);
        if (c->physics == CF2_PHYS_BULLET) {
            for (int k = 0; k < 3; ++k) E->ww[k] = F(10 + k);
            update_information(E);
        } else {
            REAL Rm[9];
            for (int k = 0; k < 3; ++k) E->wb[k] = F(10 + k);
            for (int k = 0; k < 3; ++k) E->rpy[k] = F(13 + k);
            orc_rotmat(E->q, Rm);
            matTvec(Rm, E->wb, E->ww);
        }
#undef F
        E->ep_step = si[0 * N + i];
        E->iteration = E->ep_step * c->aggregate_phy_steps;
        E->rng_ctr = (uint32_t)si[1 * N + i];
        int fl = si[2 * N + i];
        E->aidx = fl & 15;
        E->halias[0] = (fl >> 4) & 1;
        E->halias[1] = (fl >> 5) & 1;
        E->last_action_is_view = (fl >> 6) & 1;
        E->props_on = (fl >> 7) & 1;
        for (int k = 0; k < 4; ++k) E->last_action[k] = E->abuf[c->buf_size - 1][k];
        E->level_idx = si[3 * N + i];
        E->gust_left = si[4 * N + i];
    }
}
int orc_num_fields(int which) { return which == 0 ? NF : NI; }

/* ---- component entry points for golden-vector tests (REAL-typed via double I/O) ---- */
void orc_t_rotmat(const double* q, double* Rm) { REAL a[4], o[9]; for (int k = 0; k < 4; ++k) a[k] = R(q[k]); orc_rotmat(a, o); for (int k = 0; k < 9; ++k) Rm[k] = o[k]; }
void orc_t_quat_from_euler(const double* e, double* q) { REAL a[3], o[4]; for (int k = 0; k < 3; ++k) a[k] = R(e[k]); orc_quat_from_euler(a, o); for (int k = 0; k < 4; ++k) q[k] = o[k]; }
void orc_t_euler_from_quat(const double* q, double* e) { REAL a[4], o[3]; for (int k = 0; k < 4; ++k) a[k] = R(q[k]); orc_euler_from_quat(a, o); for (int k = 0; k < 3; ++k) e[k] = o[k]; }
void orc_t_quat2euler(const double* q, double* e) { REAL a[4], o[3]; for (int k = 0; k < 4; ++k) a[k] = R(q[k]); orc_quat2euler(a, o); for (int k = 0; k < 3; ++k) e[k] = o[k]; }
/* batched distur_gener (double states in, as the reference passes them) */
void orc_t_hj(const cf2_config* cfg, const float* V, const double* states, int n, double level,
              double* dopt, double* uopt, int32_t* idx) {
    for (int i = 0; i < n; ++i)
        orc_hj_eval(cfg, V, states + 6 * i, level, dopt + 3 * i, uopt + 3 * i, idx ? idx + 6 * i : NULL);
}
/* apply_action sequence on one fresh agent: acts [T,4], ou_normals [T,4] -> forces [T,4], tz [T], x [T,4] */
void orc_t_apply_action(const cf2_config* cfg, int T, const double* acts, const double* ou_n,
                        const double* init_x, const double* init_buf, double* forces, double* tz, double* xs) {
    orc_ctx X; memset(&X, 0, sizeof(X)); X.cfg = *cfg;
    orc_env E; memset(&E, 0, sizeof(E));
    for (int j = 0; j < 4; ++j) { E.A[j] = R(cfg->A); E.B[j] = R(cfg->B); E.K[j] = R(cfg->K); E.x[j] = R(init_x[j]); }
    for (int r = 0; r < cfg->buf_size; ++r) for (int j = 0; j < 4; ++j) E.abuf[r][j] = R(init_buf[4 * r + j]);
    E.k0 = R(cfg->ft0); E.k1 = R(cfg->ft1);
    for (int t = 0; t < T; ++t) {
        REAL a[4], n[4], f[4], z;
        for (int j = 0; j < 4; ++j) { a[j] = R(acts[4 * t + j]); n[j] = R(ou_n[4 * t + j]); }
        apply_action(&X, &E, a, n, f, &z);
        for (int j = 0; j < 4; ++j) { forces[4 * t + j] = f[j]; xs[4 * t + j] = E.x[j]; }
        tz[t] = z;
    }
}
/* SensorNoise.add_noise given recorded normals n[18] (pos,vel,bias,rw,turn-on,rot) and
 * uniforms uu[6] in [0,1) (pos, rot) -> pos, vel, rot, omega; bias in/out */
void orc_t_add_noise(const cf2_config* cfg, const double* pos, const double* vel, const double* rot,
                     const double* omega, const double* n, const double* uu, double* bias,
                     double* opos, double* ovel, double* orot, double* oomega) {
    orc_env E; memset(&E, 0, sizeof(E));
    for (int k = 0; k < 3; ++k) E.bias[k] = R(bias[k]);
    REAL nn[18], w[3], om[3];
    for (int k = 0; k < 18; ++k) nn[k] = R(n[k]);
    for (int k = 0; k < 3; ++k) w[k] = R(omega[k]);
    for (int k = 0; k < 3; ++k) {
        REAL uo = R(-cfg->pos_unif_range) + (R(cfg->pos_unif_range) - R(-cfg->pos_unif_range)) * R(uu[k]);
        opos[k] = R(pos[k]) + (R(cfg->pos_norm_std) * nn[k] + uo);
        ovel[k] = R(vel[k]) + R(cfg->vel_norm_std) * nn[3 + k] + R(0.0);
    }
    omega_noise(cfg, &E, w, nn + 6, om);
    const REAL lo[3] = {R(-3.141592653589793), R(-1.5707963267948966), R(-3.141592653589793)};
    for (int k = 0; k < 3; ++k) {
        REAL uo = R(-cfg->rot_unif_range) + (R(cfg->rot_unif_range) - R(-cfg->rot_unif_range)) * R(uu[3 + k]);
        REAL th = R(cfg->rot_norm_std) * nn[15 + k] + uo;
        orot[k] = clampr(R(rot[k]) + th, lo[k], -lo[k]);
    }
    for (int k = 0; k < 3; ++k) { oomega[k] = om[k]; bias[k] = E.bias[k]; }
}
/* one bullet sub-step on a single env given explicit state (for known-answer tests) */
void orc_t_bullet_substep(const cf2_config* cfg, double* st /* p3 q4 v3 ww3 x4 ou4 abuf8 */,
                          const double* a, const double* dstb, const double* ou_n, int first_after_reset,
                          double* out_rpy_wb /* 6 */) {
    orc_ctx X; memset(&X, 0, sizeof(X)); X.cfg = *cfg;
    orc_env E; memset(&E, 0, sizeof(E));
    for (int k = 0; k < 3; ++k) { E.p[k] = R(st[k]); E.v[k] = R(st[7 + k]); E.ww[k] = R(st[10 + k]); }
    for (int k = 0; k < 4; ++k) { E.q[k] = R(st[3 + k]); E.x[k] = R(st[13 + k]); E.ou[k] = R(st[17 + k]); }
    for (int r = 0; r < 2; ++r) for (int k = 0; k < 4; ++k) E.abuf[r][k] = R(st[21 + 4 * r + k]);
    E.dt = R(cfg->time_step); E.m = R(cfg->mass); E.J[0] = R(cfg->ixx); E.J[1] = R(cfg->iyy); E.J[2] = R(cfg->izz);
    E.k0 = R(cfg->ft0); E.k1 = R(cfg->ft1);
    for (int j = 0; j < 4; ++j) { E.A[j] = R(cfg->A); E.B[j] = R(cfg->B); E.K[j] = R(cfg->K); }
    REAL aa[4], dd[3], nn[4];
    for (int k = 0; k < 4; ++k) { aa[k] = R(a[k]); nn[k] = R(ou_n[k]); }
    for (int k = 0; k < 3; ++k) dd[k] = R(dstb[k]);
    bullet_substep(&X, &E, aa, dd, nn, first_after_reset, R(0.0));
    for (int k = 0; k < 3; ++k) { st[k] = E.p[k]; st[7 + k] = E.v[k]; st[10 + k] = E.ww[k]; }
    for (int k = 0; k < 4; ++k) { st[3 + k] = E.q[k]; st[13 + k] = E.x[k]; st[17 + k] = E.ou[k]; }
    for (int r = 0; r < 2; ++r) for (int k = 0; k < 4; ++k) st[21 + 4 * r + k] = E.abuf[r][k];
    for (int k = 0; k < 3; ++k) { out_rpy_wb[k] = E.rpy[k]; out_rpy_wb[3 + k] = E.wb[k]; }
}
/* SimplePhysics step given explicit drone attributes (pos3 quat4 rpy3 vel3 rate3) */
void orc_t_simple_substep(const cf2_config* cfg, double* st, const double* a, const double* ou_n, double* ou) {
    orc_ctx X; memset(&X, 0, sizeof(X)); X.cfg = *cfg;
    orc_env E; memset(&E, 0, sizeof(E));
    for (int k = 0; k < 3; ++k) { E.p[k] = R(st[k]); E.rpy[k] = R(st[7 + k]); E.v[k] = R(st[10 + k]); E.wb[k] = R(st[13 + k]); }
    for (int k = 0; k < 4; ++k) { E.q[k] = R(st[3 + k]); E.ou[k] = R(ou[k]); }
    E.dt = R(cfg->time_step); E.m = R(cfg->mass); E.J[0] = R(cfg->ixx); E.J[1] = R(cfg->iyy); E.J[2] = R(cfg->izz);
    E.k0 = R(cfg->ft0); E.k1 = R(cfg->ft1);
    for (int j = 0; j < 4; ++j) { E.A[j] = R(cfg->A); E.B[j] = R(cfg->B); E.K[j] = R(cfg->K); }
    REAL aa[4], nn[4];
    for (int k = 0; k < 4; ++k) { aa[k] = R(a[k]); nn[k] = R(ou_n[k]); }
    simple_substep(&X, &E, aa, nn);
    for (int k = 0; k < 3; ++k) { st[k] = E.p[k]; st[7 + k] = E.rpy[k]; st[10 + k] = E.v[k]; st[13 + k] = E.wb[k]; }
    for (int k = 0; k < 4; ++k) { st[3 + k] = E.q[k]; ou[k] = E.ou[k]; }
}
/* reward / done / cost on explicit attributes: attrs = p3 rpy3 v3 wb3 last_action4 */
void orc_t_reward_done_cost(const cf2_config* cfg, const double* attrs, const double* a,
                            double* r, int* done, double* cost) {
    orc_env E; memset(&E, 0, sizeof(E));
    for (int k = 0; k < 3; ++k) { E.p[k] = R(attrs[k]); E.rpy[k] = R(attrs[3 + k]); E.v[k] = R(attrs[6 + k]); E.wb[k] = R(attrs[9 + k]); }
    for (int k = 0; k < 4; ++k) E.last_action[k] = R(attrs[12 + k]);
    REAL aa[4];
    for (int k = 0; k < 4; ++k) aa[k] = R(a[k]);
    int d = compute_done(cfg, &E);
    *done = d;
    *r = (double)compute_reward(cfg, &E, aa, d);
    *cost = (double)compute_cost(cfg, &E);
}
int orc_t_boltzmann_index(const cf2_config* cfg, double u) { return boltzmann_index(cfg, R(u)); }
