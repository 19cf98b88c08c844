/* asan_driver.c -- TEST INFRASTRUCTURE ONLY: drives the CPU restatement (cf2_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (`make asan`, tests/test_oracle_asan.py).
 * usage: asan_driver CONFIG_BLOB STEPS
 * CONFIG_BLOB holds one cf2_config exactly as cf2sim.config.build_config lays it out (the test
 * writes it with ctypes); the driver exercises reset, env-steps with every optional output,
 * masked reset, the physics plug-in step, the snapshot round trip and, for HJ envs, a synthetic
 * 15^6 table per level. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../include/cf2sim.h"

void* orc_create(const cf2_config* cfg);
void orc_destroy(void* h);
void orc_bind_tables(void* h, const float* V, int num_tables, const int32_t* table_of_level);
void orc_reset(void* h, const uint8_t* mask, double* obs);
void orc_step(void* h, const float* act, const double* dstb_ext, double* obs, double* rew, uint8_t* done_out,
              uint8_t* trunc_out, double* cost_out, double* level_out, double* final_obs);
void orc_physics_step(void* h, const float* act, const double* dstb, double dt_override);
void orc_get_state(void* h, double* sf, int32_t* si);
void orc_set_state(void* h, const double* sf, const int32_t* si);
int orc_num_fields(int which);

static uint32_t lcg(uint32_t* s) { *s = *s * 1664525u + 1013904223u; return *s; }
static float unif(uint32_t* s) { return (float)(lcg(s) >> 8) * (2.0f / 16777216.0f) - 1.0f; }

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s CONFIG_BLOB STEPS\n", argv[0]); return 2; }
    cf2_config cfg;
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror("config"); return 2; }
    if (fread(&cfg, 1, sizeof(cfg), f) != sizeof(cfg) || fgetc(f) != EOF) { fprintf(stderr, "config size mismatch\n"); return 2; }
    fclose(f);
    const int steps = atoi(argv[2]);
    const size_t n = cfg.num_envs;
    const int od = cfg.observation_noise_on ? 34 : 42;
    void* h = orc_create(&cfg);
    float* V = NULL;
    if (cfg.disturbance == CF2_DSTB_HJ) {
        const size_t cells = (size_t)11390625;
        const int T = 2;
        V = (float*)malloc(sizeof(float) * cells * T);
        uint32_t s = 7;
        for (size_t k = 0; k < cells * T; ++k) V[k] = unif(&s);
        int32_t tol[CF2_NUM_LEVELS_MAX];
        for (int l = 0; l < CF2_NUM_LEVELS_MAX; ++l) tol[l] = l % T;
        orc_bind_tables(h, V, T, tol);
    }
    double* obs = (double*)malloc(sizeof(double) * n * od);
    double* fin = (double*)malloc(sizeof(double) * n * od);
    double* rew = (double*)malloc(sizeof(double) * n);
    double* cost = (double*)malloc(sizeof(double) * n);
    double* level = (double*)malloc(sizeof(double) * n);
    double* dstb = (double*)malloc(sizeof(double) * n * 3);
    uint8_t* done = (uint8_t*)malloc(n);
    uint8_t* trunc = (uint8_t*)malloc(n);
    uint8_t* mask = (uint8_t*)malloc(n);
    float* act = (float*)malloc(sizeof(float) * n * 4);
    uint32_t s = 12345;
    orc_reset(h, NULL, obs);
    size_t dones = 0;
    for (int t = 0; t < steps; ++t) {
        for (size_t k = 0; k < n * 4; ++k) act[k] = unif(&s);
        for (size_t k = 0; k < n * 3; ++k) dstb[k] = 1e-4 * unif(&s);
        orc_step(h, act, cfg.disturbance == CF2_DSTB_EXTERNAL ? dstb : NULL, obs, rew, done, trunc, cost, level,
                 (t & 1) ? fin : NULL);
        for (size_t i = 0; i < n; ++i) dones += done[i];
    }
    for (size_t i = 0; i < n; ++i) mask[i] = (uint8_t)(i % 3 == 0);
    orc_reset(h, mask, obs);
    for (int t = 0; t < 4; ++t) orc_physics_step(h, act, (t & 1) ? dstb : NULL, (t & 2) ? 0.004 : 0.0);
    const int nf = orc_num_fields(0), ni = orc_num_fields(1);
    double* sf = (double*)malloc(sizeof(double) * n * (size_t)nf);
    int32_t* si = (int32_t*)malloc(sizeof(int32_t) * n * (size_t)ni);
    orc_get_state(h, sf, si);
    orc_set_state(h, sf, si);
    orc_step(h, act, cfg.disturbance == CF2_DSTB_EXTERNAL ? dstb : NULL, obs, rew, done, NULL, NULL, NULL, NULL);
    double chk = 0.0;
    for (size_t k = 0; k < n * od; ++k) chk += obs[k];
    printf("ok envs=%zu steps=%d dones=%zu checksum=%.6e\n", n, steps, dones, chk);
    free(sf); free(si); free(obs); free(fin); free(rew); free(cost); free(level); free(dstb);
    free(done); free(trunc); free(mask); free(act); free(V);
    orc_destroy(h);
    return 0;
}
