/*
 * gpd.h — C ABI of the MI355X-native batched quadrotor DYN path.
 *
 * This is the drop-in boundary for the reference's hot path (paths relative to the
 * reference root, gym_pybullet_drones/):
 *
 *   gpd_create        <- BaseAviary.__init__            envs/BaseAviary.py:25-216
 *                        (+ _parseURDFParameters :982-1014, derived constants :117-128,
 *                           BaseRLAviary.__init__ action buffer envs/BaseRLAviary.py:66-67,
 *                           HoverAviary TARGET_POS/EPISODE_LEN_SEC envs/HoverAviary.py:51-52,
 *                           MultiHoverAviary TARGET_POS envs/MultiHoverAviary.py:71)
 *   gpd_reset         <- BaseAviary.reset()             envs/BaseAviary.py:220-255
 *                        (+ _housekeeping :451-505, readback :509-519, _computeObs
 *                           envs/BaseRLAviary.py:284-319)
 *   gpd_step          <- BaseAviary.step()              envs/BaseAviary.py:259-383, i.e.
 *                        _preprocessAction (BaseRLAviary.py:160-239; the PID types run
 *                        DSLPIDControl, control/DSLPIDControl.py:82-259),
 *                        PYB_STEPS_PER_CTRL x (_updateAndStoreKinematicInformation :509-519
 *                        + _dynamics :815-874 + _integrateQ :876-889
 *                        [+ _groundEffect :715-750, _drag :754-781, _downwash :785-811]),
 *                        _computeObs / _computeReward / _computeTerminated /
 *                        _computeTruncated (HoverAviary.py:68-117, MultiHoverAviary.py:75-130),
 *                        plus SB3 VecEnv auto-reset (optional).
 *   gpd_integrate     <- the raw _dynamics + readback substep (:815-889, :509-519) driven by
 *                        explicit per-substep RPMs (parity / raw-integrator mode).
 *   gpd_get_state20   <- BaseAviary._getDroneStateVector()  envs/BaseAviary.py:541-561
 *   gpd_set_pid_params <- BaseControl.setPIDCoefficients()   control/BaseControl.py:138-177
 *   gpd_get/set_ctrl_state <- the per-drone DSLPIDControl attributes integral_pos_e,
 *                        integral_rpy_e, last_rpy (control/DSLPIDControl.py:65-78)
 *   gpd_pack_layout_of / gpd_handoff_pack / gpd_handoff_unpack <- the hand-off of the
 *                        vectorised step to the learner across GPUs (the caller SB3 runs in one
 *                        process in examples/learn.py:52-94): obs, reward, dones and
 *                        infos["terminal_observation"] of every rank's env shard
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (hipMalloc'd memory, e.g. a torch tensor's
 *     data_ptr()) unless named *_host.  The caller owns every I/O buffer; the sim owns its
 *     state.  No call allocates or synchronises except gpd_create / gpd_destroy /
 *     gpd_save_state / gpd_load_state.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  All work is
 *     enqueued asynchronously on it.  Calls on one handle must be serialised by the caller.
 *   - Drones are numbered env-major: drone n = env * drones_per_env + d.
 *   - "real" below is float (GPD_F32) or double (GPD_F64), chosen at create time.
 *   - Return value: GPD_OK (0) or a negative GPD_E* code; gpd_last_error() describes the
 *     last failure of the calling thread.
 */
#ifndef GPD_H_
#define GPD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPD_ABI_VERSION 7

/* return codes */
#define GPD_OK 0
#define GPD_EINVAL (-1)       /* invalid argument / configuration (BaseAviary.py:79-80 ValueError) */
#define GPD_EHIP (-2)         /* HIP runtime error */
#define GPD_ENOMEM (-3)       /* device allocation failed */
#define GPD_EUNSUPPORTED (-4) /* valid in the reference, not on this path (e.g. RGB obs) */

/* DroneModel (utils/enums.py:3-8) */
#define GPD_MODEL_CF2X 0
#define GPD_MODEL_CF2P 1
#define GPD_MODEL_RACE 2

/* ActionType (utils/enums.py:35-41; BaseRLAviary._preprocessAction :160-239) */
#define GPD_ACT_RPM 0         /* width 4: rpm = HOVER_RPM*(1+0.05a)                 :191-192 */
#define GPD_ACT_ONE_D_RPM 1   /* width 1: same, repeated on the 4 motors            :224-225 */
#define GPD_ACT_PID 2         /* width 3: DSLPIDControl to _calculateNextStep(pos, a, 1) :193-207 */
#define GPD_ACT_VEL 3         /* width 4: DSLPIDControl to velocity SPEED_LIMIT*|a3|*a/|a| :208-223 */
#define GPD_ACT_ONE_D_PID 4   /* width 1: DSLPIDControl to pos + (0,0,0.1a)         :226-235 */

/* Task hooks (reward / terminated / truncated) */
#define GPD_TASK_NONE 0       /* raw aviary: reward -1, never done (CtrlAviary-like) */
#define GPD_TASK_HOVER 1      /* HoverAviary.py:68-117 */
#define GPD_TASK_MULTIHOVER 2 /* MultiHoverAviary.py:75-130 */

/* physics flags: force terms added to the explicit integrator (Physics enum utils/enums.py:13-21) */
#define GPD_F_GND 1           /* _groundEffect  BaseAviary.py:715-750 */
#define GPD_F_DRAG 2          /* _drag          BaseAviary.py:754-781 */
#define GPD_F_DW 4            /* _downwash      BaseAviary.py:785-811 */
#define GPD_F_GEOM_WRENCH 8   /* prop thrust torque from URDF prop positions (_physics :679-711)
                                 instead of the DYN formula (:846-851) */
#define GPD_F_BULLET 16       /* Physics.PYB*: the forces go through a restated Bullet3 btMultiBody
                                 base step (p.stepSimulation, :369-370; default damping 0.04,
                                 world-frame angular velocity, exponential-map orientation, velocity
                                 clamp 100, ground-plane contact of the collision cylinder) instead
                                 of _dynamics; implies GEOM_WRENCH */
#define GPD_F_NO_PLANE 32     /* with GPD_F_BULLET: no drone <-> plane contact (the reference's
                                 commented-out setCollisionFilterPair, BaseAviary.py:500-503) */
#define GPD_F_NO_DRONE_CONTACT 64 /* with GPD_F_BULLET: no drone <-> drone contact between the drones
                                 of an env (on by default: every drone is a colliding Bullet body,
                                 BaseAviary.py:486-491) */

/* precision */
#define GPD_F32 0
#define GPD_F64 1

/* Drone model parameters (the URDF <properties>, inertial and prop-link values parsed by
 * BaseAviary._parseURDFParameters, BaseAviary.py:982-1014). */
typedef struct gpd_drone_params {
  int model;                 /* GPD_MODEL_* (selects the DYN torque formula, :843-851) */
  double m, arm, thrust2weight, ixx, iyy, izz, kf, km;
  double collision_h, collision_r, collision_z_offset, max_speed_kmh;
  double gnd_eff_coeff, prop_radius, drag_coeff_xy, drag_coeff_z;
  double dw_coeff_1, dw_coeff_2, dw_coeff_3;
  double prop_pos[4][3];     /* prop link inertial origins (cf2x.urdf:42,54,66,78) */
} gpd_drone_params;

typedef struct gpd_config {
  int n_envs;                /* E >= 1 */
  int drones_per_env;        /* D in [1, 1024] (HoverAviary: 1); D > 64 runs one env per multi-wave workgroup */
  int pyb_freq;              /* PYB_FREQ, default 240 */
  int ctrl_freq;             /* CTRL_FREQ, must divide pyb_freq (HoverAviary default 30) */
  int act_type;              /* GPD_ACT_* */
  int task;                  /* GPD_TASK_* */
  int physics_flags;         /* OR of GPD_F_* */
  int precision;             /* GPD_F32 or GPD_F64 */
  int autoreset;             /* 1: done envs are reset inside gpd_step (SB3 VecEnv semantics) */
  double episode_len_sec;    /* EPISODE_LEN_SEC (8 for both tasks) */
  const double* init_xyzs_host; /* [D][3] INIT_XYZS shared by all envs, NULL = default (:194-197) */
  const double* init_rpys_host; /* [D][3] INIT_RPYS, NULL = zeros */
  /* Launch tuning: 0 = automatic (the measured defaults).  Explicit values exist for A/B
   * experiments and tests; they change launch geometry and store policy, never results
   * beyond the rounding noted in DESIGN.md section 4. */
  int drones_per_block;      /* drones per step block (rounded to whole envs, <= 64) */
  int step_waves;            /* plain-DYN single-drone RPM path: 1 single-wave kernel,
                              * 2 pose+rate waves, 3 pose+rate+io waves */
  int store_policy;          /* 1 + write-through mask: bit 0 obs/terminal rows, bit 1 state */
  /* Contact solver of the PYB* modes, as pybullet's setPhysicsEngineParameter sets it
   * (numSolverIterations, solverResidualThreshold; BaseAviary.py never calls it, so the
   * defaults are the reference's): 0 = default (50 iterations, residual 1e-7); a residual < 0
   * makes every solve run all its iterations. */
  int solver_iterations;     /* 0 or [1, 1000] */
  double solver_residual;
} gpd_config;

/* Derived constants, BaseAviary.py:117-128 (read-only view for tests/facades). */
typedef struct gpd_constants {
  double gravity, hover_rpm, max_rpm, max_thrust, max_xy_torque, max_z_torque, gnd_eff_h_clip;
  double pyb_timestep, ctrl_timestep;
  int pyb_steps_per_ctrl, action_buffer_size, obs_width, act_width, n_drones;
  int trunc_step_counter;    /* smallest step_counter with step_counter/PYB_FREQ > EPISODE_LEN_SEC */
  int drones_per_block;      /* drones per block of the step kernel (launch geometry) */
  int lanes_per_block;       /* step kernel block size: 64, 128 (two waves) or 192 (three) */
} gpd_constants;

/* DSLPIDControl coefficients and constants (control/DSLPIDControl.py:37-60; GRAVITY and KF
 * from the cf2x URDF, BaseControl.py:35-39 - BaseRLAviary builds the CF2X controller for cf2x
 * and cf2p drones alike, envs/BaseRLAviary.py:75-76). */
typedef struct gpd_pid_params {
  double p_coeff_for[3], i_coeff_for[3], d_coeff_for[3];
  double p_coeff_tor[3], i_coeff_tor[3], d_coeff_tor[3];
  double pwm2rpm_scale, pwm2rpm_const, min_pwm, max_pwm;
  double mixer[4][3];
  double gravity, kf;
} gpd_pid_params;

typedef struct gpd_sim gpd_sim;

int gpd_abi_version(void);
const char* gpd_last_error(void);

/* Fill `out` with the built-in parameters of a drone model (cf2x/cf2p/racer URDF values). */
int gpd_default_params(int model, gpd_drone_params* out);

/* The DSLPIDControl(DroneModel.CF2X) defaults. */
int gpd_default_pid_params(gpd_pid_params* out);

/* Create a batched aviary on the CURRENT HIP device; state is initialised as after reset()
 * and the action ring (15 = ctrl_freq//2 slots) is zero, as BaseRLAviary._actionSpace leaves it. */
int gpd_create(const gpd_drone_params* params, const gpd_config* cfg, gpd_sim** out);
int gpd_destroy(gpd_sim* sim);
int gpd_get_constants(const gpd_sim* sim, gpd_constants* out);

/* reset(): envs with env_mask[e] != 0 (env_mask == NULL: all envs) go back to INIT_XYZS /
 * INIT_RPYS with zero velocities, step_counter 0, last_clipped_action 0.  The action ring is
 * NOT cleared (the reference never clears action_buffer).  If obs != NULL the reset
 * observation rows [E][D][obs_width] float of the reset envs are written. */
int gpd_reset(gpd_sim* sim, const uint8_t* env_mask, float* obs, void* stream);

/* step(action): actions [E][D][act_width] float in, obs [E][D][obs_width] float,
 * reward [E] float, terminated/truncated [E] uint8 out.  With autoreset, done envs are reset
 * after their terminal row is copied to terminal_obs [E][D][obs_width] (if non-NULL; rows of
 * envs that are not done are left untouched) and obs holds the reset observation. */
int gpd_step(gpd_sim* sim, const float* actions, float* obs, float* reward,
             uint8_t* terminated, uint8_t* truncated, float* terminal_obs, void* stream);

/* n_steps consecutive gpd_step calls issued from native code (open-loop action sequences:
 * playback, benchmarks): step t reads action slot t % n_slots of actions
 * [n_slots][E][D][act_width]; every step writes the same output buffers (as n_steps gpd_step
 * calls would), so they hold the last step's outputs.  One kernel launch per step, no host
 * round trip in between. */
int gpd_step_seq(gpd_sim* sim, const float* actions, int n_slots, int n_steps, float* obs, float* reward,
                 uint8_t* terminated, uint8_t* truncated, float* terminal_obs, void* stream);

/* Raw DYN integrator: n_sub substeps, row t of rpm [n_sub][N][4] (real) drives substep t of
 * every drone; each substep is followed by the readback (PYB_STEPS_PER_CTRL = 1 cadence).
 * traj (nullable) receives the 20-float state after every substep, [n_sub][N][20] real. */
int gpd_integrate(gpd_sim* sim, const void* rpm, int n_sub, void* traj, void* stream);

/* 20-float state vectors [N][20] real (BaseAviary.py:541-561). */
int gpd_get_state20(gpd_sim* sim, void* out, void* stream);

/* Raw per-drone state [N][20] real = pos(3) quat_xyzw as stored by the physics client (4)
 * vel(3) rpy_rates(3) ang_v_world(3) last_clipped_action(4).  Used for checkpoints and to
 * seed arbitrary initial conditions. */
int gpd_get_raw_state(gpd_sim* sim, void* out, void* stream);
int gpd_set_raw_state(gpd_sim* sim, const void* in, void* stream);
/* Per-env non-finite guard (new, the reference has none): env_flags [E] uint8
 * (device memory) = 1 where any drone of the env holds a non-finite pos / quat / vel / rate /
 * ang_v component (e.g. the downwash quotient at beta = 0, BaseAviary.py:802-804), else 0.
 * Asynchronous on `stream`; the step path itself never tests for it. */
int gpd_nonfinite(gpd_sim* sim, uint8_t* env_flags, void* stream);
/* PID action types: replace the controller coefficients of every drone (setPIDCoefficients).
 * Synchronous (uploads the constant block). */
int gpd_set_pid_params(gpd_sim* sim, const gpd_pid_params* params);
/* PID action types: per-drone controller state [N][9] real = integral_pos_e(3)
 * integral_rpy_e(3) last_rpy(3).  Zero at create; NOT cleared by gpd_reset (the reference
 * never resets its controllers after construction). */
int gpd_get_ctrl_state(gpd_sim* sim, void* out, void* stream);
int gpd_set_ctrl_state(gpd_sim* sim, const void* in, void* stream);
/* step counters [E] int32 */
int gpd_get_step_counters(gpd_sim* sim, int32_t* out, void* stream);
int gpd_set_step_counters(gpd_sim* sim, const int32_t* in, void* stream);

/* Whole-sim checkpoint (state, controller state, action ring, ring head, step counters) to/from host memory.
 * gpd_state_bytes gives the blob size (the caller's buffer must have exactly that size); the
 * blob's 64-byte header (ABI version, N, E, D, action type, precision, ring length, padding)
 * must match the loading sim, else GPD_EINVAL.  These synchronise `stream`. */
size_t gpd_state_bytes(const gpd_sim* sim);
int gpd_save_state(gpd_sim* sim, void* blob_host, void* stream);
int gpd_load_state(gpd_sim* sim, const void* blob_host, void* stream);

/* ---- Config-5 learner hand-off.  Replaces the reference's stepping loop
 * examples/learn.py:52-94, where SB3 steps one process's VecEnv and hands obs / reward / done /
 * infos["terminal_observation"] to PPO.  Here each rank (one per GPU) steps its env shard into
 * one output pack; one collective moves every rank's RECORD = [obs | reward | terminated |
 * truncated | terminal_state] to the learner; gpd_handoff_unpack rebuilds the global batch.
 *
 * Pack layout of a shard of E envs x D drones, obs rows of W floats (every field 256-B aligned,
 * offsets in bytes):  obs [E][D][W] f32 | reward [E] f32 | terminated [E] u8 | truncated [E] u8 |
 * terminal_state [E][D][12] f32 | terminal_obs [E][D][W] f32.  gpd_step writes obs, reward, the
 * flags and terminal_obs into their fields; gpd_handoff_pack fills terminal_state. */
typedef struct gpd_pack_layout {
  int n_envs, drones_per_env, obs_width, state_cols; /* state_cols = 12 (pos, rpy, vel, ang_v) */
  long long obs, reward, terminated, truncated, terminal_state, terminal_obs;
  long long prefix;          /* end of the truncated flags */
  long long prefix_aligned;  /* prefix rounded up to 256: a record without terminal rows */
  long long record;          /* end of terminal_state (256-aligned): one rank's hand-off record */
  long long total;           /* bytes of the whole pack */
} gpd_pack_layout;

int gpd_pack_layout_of(int n_envs, int drones_per_env, int obs_width, gpd_pack_layout* out);

/* Before the exchange: for every env whose terminated or truncated flag is set in `pack`, copy
 * columns 0..11 of its terminal_obs rows into terminal_state (other envs' entries are left
 * as they are: the unpack never reads them).  The reference never clears the action buffer on
 * reset (BaseRLAviary.py has no reset override), so a finished env's terminal row and its
 * auto-reset row share the history columns: the receivers rebuild the whole row. */
int gpd_handoff_pack(uint8_t* pack, const gpd_pack_layout* layout, void* stream);

/* After the exchange: `gathered` holds n_ranks records, `stride` bytes apart (layout->record, or
 * layout->prefix_aligned when no terminal rows travelled).  Writes the global batch in rank
 * order: obs [n_ranks*E][D][W], reward [n_ranks*E], terminated / truncated [n_ranks*E] and, when
 * terminal_obs != NULL (needs stride = record), the terminal rows [n_ranks*E][D][W]: for a
 * finished env its 12 state columns followed by the gathered obs row's history columns, zero for
 * every other env (infos[i]["terminal_observation"] of SB3's DummyVecEnv). */
int gpd_handoff_unpack(const uint8_t* gathered, int n_ranks, long long stride, const gpd_pack_layout* layout,
                       float* obs, float* reward, uint8_t* terminated, uint8_t* truncated, float* terminal_obs,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GPD_H_ */
