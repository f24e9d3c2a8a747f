/* AddressSanitizer / UBSan drive of the C restatement (TEST INFRASTRUCTURE ONLY, SURVEY.md §5:
 * "an ASan build of the C oracle"): the whole translation unit is compiled into this program with
 * -fsanitize=address,undefined (oracle/Makefile target `asan`) and every public entry point is
 * exercised on the shapes the tests use - single- and 8-drone envs, every force-term flag, both
 * action widths, auto-reset with terminal rows, the raw integrator with a trajectory.  Exit 0 and
 * no sanitizer report = clean (tests/test_c_oracle.py::test_oracle_under_asan). */
#include "gpd_oracle.c"

#include <stdio.h>

static void cf2x(orc_params* p) {
  memset(p, 0, sizeof(*p));
  p->model = 0; p->m = 0.027; p->arm = 0.0397; p->thrust2weight = 2.25;
  p->ixx = 1.4e-5; p->iyy = 1.4e-5; p->izz = 2.17e-5; p->kf = 3.16e-10; p->km = 7.94e-12;
  p->collision_h = 0.025; p->collision_r = 0.06; p->collision_z_offset = 0.0;
  p->gnd_eff_coeff = 11.36859; p->prop_radius = 2.31348e-2;
  p->drag_coeff_xy = 9.1785e-7; p->drag_coeff_z = 10.311e-7;
  p->dw1 = 2267.18; p->dw2 = 0.16; p->dw3 = -0.11;
  const double pp[4][3] = {{0.028, -0.028, 0}, {-0.028, -0.028, 0}, {-0.028, 0.028, 0}, {0.028, 0.028, 0}};
  memcpy(p->prop_pos, pp, sizeof(pp));
}

static unsigned rng_state = 12345u;
static float urand(void) {   /* U[-1, 1) */
  rng_state = rng_state * 1664525u + 1013904223u;
  return (float)((rng_state >> 8) * (1.0 / 16777216.0)) * 2.0f - 1.0f;
}

static int run(int E, int D, int A, int task, int flags, int steps) {
  orc_params p;
  cf2x(&p);
  double xyz[8 * 3];
  for (int d = 0; d < D; ++d) {
    xyz[3 * d] = 0.15 * cos(0.785 * d); xyz[3 * d + 1] = 0.15 * sin(0.785 * d); xyz[3 * d + 2] = 0.5 + 0.1 * d;
  }
  orc_sim* S = orc_create(&p, E, D, 240, 30, A, task, flags, 1, 8.0, D > 1 ? xyz : NULL, NULL);
  if (!S) return 1;
  const int N = E * D, W = orc_obs_width(S);
  float* act = (float*)malloc(sizeof(float) * N * A);
  float* obs = (float*)malloc(sizeof(float) * N * W);
  float* tobs = (float*)malloc(sizeof(float) * N * W);
  float* rew = (float*)malloc(sizeof(float) * E);
  uint8_t* te = (uint8_t*)malloc(E);
  uint8_t* tr = (uint8_t*)malloc(E);
  double* s20 = (double*)malloc(sizeof(double) * N * 20);
  orc_reset(S, obs);
  for (int t = 0; t < steps; ++t) {
    for (int i = 0; i < N * A; ++i) act[i] = urand();
    orc_step(S, act, obs, rew, te, tr, tobs, 2);
  }
  orc_get_state20(S, s20);
  double* raw = (double*)malloc(sizeof(double) * N * 20);
  orc_get_raw(S, raw);
  orc_set_raw(S, raw);
  const int T = 16;
  double* rpm = (double*)malloc(sizeof(double) * T * N * 4);
  double* traj = (double*)malloc(sizeof(double) * T * N * 20);
  for (int i = 0; i < T * N * 4; ++i) rpm[i] = orc_hover_rpm(S) * (1.0 + 0.05 * urand());
  orc_integrate(S, rpm, T, traj, 2);
  orc_integrate(S, rpm, T, NULL, 1);
  double chk = 0;
  for (int i = 0; i < N * 20; ++i) chk += s20[i];
  for (int i = 0; i < T * N * 20; ++i) chk += traj[i];
  printf("E=%d D=%d A=%d task=%d flags=%d: checksum %.6e\n", E, D, A, task, flags, chk);
  free(act); free(obs); free(tobs); free(rew); free(te); free(tr); free(s20); free(raw); free(rpm); free(traj);
  orc_destroy(S);
  return 0;
}

int main(void) {
  int rc = 0;
  rc |= run(8, 1, 4, TASK_HOVER, 0, 120);
  rc |= run(8, 1, 1, TASK_HOVER, F_GND | F_DRAG, 120);
  rc |= run(4, 8, 4, TASK_MULTI, F_GND | F_DRAG | F_DW, 60);
  rc |= run(3, 8, 4, TASK_NONE, F_DW | F_GEOM, 30);
  printf(rc ? "FAILED\n" : "OK\n");
  return rc;
}
