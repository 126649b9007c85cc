/*
 * astro_step.h -- C-ABI of libastro_hip.so, the MI355X (gfx950) batched
 * lockstep implementation of Astro's per-tick physics.
 *
 * The reference (DouglasOrr/Astro) has no FFI: its hot path is the Python
 * function API of astro/core.py.  Each entry point below replaces one
 * reference interface, batched over n_env independent games:
 *
 *   astro_step         <- core.step(state, control, config)  core.py:215-303
 *   astro_step_many    <- k calls of core.step with controls known ahead
 *   astro_rollout      <- core.play's tick loop with Bots.control (core.py:359-410)
 *                         for open-loop / scripted controls, K ticks per launch
 *                         (plus auto-reset = core.create(next config of the
 *                         env's generate_configs stream), core.py:77-135)
 *   astro_controls     <- core.Bots.control(bots, state)      core.py:359-363
 *                         with script.NothingBot / ScriptBot  script.py:6-91
 *   astro_reset        <- core.create(config)                 core.py:86-135
 *   astro_stream_init  <- core.generate_configs(config)       core.py:77-83
 *   astro_features     <- rl.ValueNetwork.get_features(state) + to_batch
 *                         (rl.py:36-112), the observation a policy consumes
 *   astro_game_step    <- core.step for ONE game as server.py's game_tick calls it
 *                         (server.py:41-51): state in, next state out, one call
 *
 * Conventions
 *   - The caller owns all memory the entry points read and write (e.g.
 *     PyTorch tensors): astro_step/rollout/reset/... never allocate, free or
 *     synchronise.  The only allocating calls are the optional helpers
 *     astro_host_alloc / astro_dev_alloc (and their frees), which hand the
 *     caller memory of a particular kind to own.
 *   - Every call is stream-ordered and asynchronous on `stream` (a
 *     hipStream_t passed as void*, NULL = the null stream).
 *   - Return 0 on success, a negative code on a bad argument (-1..-99) or a
 *     launch failure (-1000 - hipError_t).  astro_last_error() describes the
 *     last failure of the calling thread.
 *   - Ships and planets are struct-of-arrays, entity-major: slot s of env i
 *     lives at [s * n_env + i], so consecutive lanes (envs) touch consecutive
 *     bytes; bullets are one contiguous row per env.  Element type is float
 *     (state_f64 = 0) or double (state_f64 = 1).
 */
#ifndef ASTRO_STEP_H
#define ASTRO_STEP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ASTRO_ABI_VERSION 21

/* Physics constants: the reference Config (core.py:20-41) reduced by the
 * host exactly as the reference evaluates it, plus the fire/timeout
 * schedule of its float64 t/reload bookkeeping (core.py:257-302). */
typedef struct AstroParams {
    double gm;             /* gravity * planet_mass                 core.py:151 */
    double dt;             /* dt                                    core.py:189 */
    double db;             /* dt * ship_rspeed                      core.py:239 */
    double thrust;         /* ship_thrust                           core.py:234 */
    double r2_ss;          /* (ship_radius + ship_radius)^2         core.py:211 */
    double r2_sp;          /* (ship_radius + planet_radius)^2 */
    double r2_s0;          /* ship_radius^2   (ship <-> bullet) */
    double r2_p0;          /* planet_radius^2 (planet <-> bullet) */
    double gravity;        /* create(): planet orbital speed        core.py:121 */
    double planet_mass;
    float spawn_off;       /* float32(1.001 * ship_radius)          core.py:273 */
    float bullet_speed;    /* float32(bullet_speed)                 core.py:277 */
    float timeout_reward;  /* 1 if solo else 0                      core.py:260 */
    float outer_pos;       /* float32(outer_ship_position)          core.py:93 */
    float inner_pos;       /* float32(inner_ship_position)          core.py:95 */
    float planet_orbit;    /* float32(planet_orbit)                 core.py:119 */
    int32_t nships;        /* 1 (solo) or 2 */
    int32_t solo;
    int32_t max_planets;   /* create(): 1..max_planets planets */
    int32_t p_pad;         /* planet slots per env, 1..16 (>= max_planets) */
    int32_t b_cap;         /* bullet slots per env, 1..65535 */
    int32_t timeout_tick;  /* first tick k with max_time <= t_k + dt */
    const uint32_t *fire_bits; /* device: bit k = fire on tick k, k < timeout_tick */
    int32_t kernel;        /* ASTRO_KERNEL_AUTO / _LANE / _QUAD / _PAIR (results are identical) */
    int32_t planets_only;  /* 0, or P: an env's games are its generate_configs stream
                              (core.py:77-83) filtered to the seeds whose create()
                              draws P planets; max_planets must be a power of two
                              (one MT word decides), needs key_table for speed */
    const uint32_t *key_table; /* device, optional: key[397] of MT19937 init_genrand for
                                  every seed < 2^30 (astro_keytable_build); NULL = the
                                  397-step chain at each create (~9 us per lane) */
} AstroParams;

/* Step kernel variants.  LANE: one lane per env (64 envs per wave64).  QUAD:
 * four lanes per env (16 envs per wave) for ships and planets, and the wave's
 * live bullets spread densely over its 64 lanes; PAIR: the same with two
 * lanes per env (32 envs per wave).  QUAD and PAIR exist for p_pad <= 8:
 * larger p_pad always runs LANE.  AUTO picks LANE for p_pad > 8, else
 * QUAD for n_env <= ASTRO_QUAD_MAX_ENVS and PAIR above (measured crossover).
 * All give identical results. */
enum { ASTRO_KERNEL_AUTO = 0, ASTRO_KERNEL_LANE = 1, ASTRO_KERNEL_QUAD = 2, ASTRO_KERNEL_PAIR = 3 };
#define ASTRO_QUAD_MAX_ENVS 32768

/* Per-env state arrays (device pointers).  hdr packs
 *   hdr[4*i+0] = tick (steps since create, < 2^22)
 *   hdr[4*i+1] = nplanets | flags << 8 | nbullets << 16
 *   hdr[4*i+2] = the NEXT game's seed (drawn one game ahead from the stream,
 *                < 2^30) | key_valid << 31, or undrawn << 30 alone: a game's
 *                create leaves the draw to its first step, off the reset path
 *   hdr[4*i+3] = key[397] of that seed's MT19937 init chain (when key_valid)
 * flags: bit0 = a bullet was dropped (b_cap full) this game,
 *        bit1 = create() needed more than 227 words of its seed's MT19937
 *               (masked randint rejections; unreachable in practice).
 * A running step fetches the next game's key[397] from the key table once,
 * so an auto-reset never runs the 397-step chain inline. */
typedef struct AstroState {
    void *ships;        /* [nships][n_env][4]  x, y, dx, dy */
    void *ships_b;      /* [nships][n_env]     bearing */
    void *planets;      /* [p_pad][n_env][4]   x, y, dx, dy */
    void *bullets;      /* [n_env][b_cap][4]   x, y, dx, dy (one contiguous row per env) */
    int32_t *hdr;       /* [n_env][4], 16-byte aligned */
    uint32_t *stream;   /* [n_env][4] generate_configs cursor: x_k, x_{k+397}, k, current game's seed
                           (x = the MT19937 word sequence of the env's RandomState, core.py:79) */
    uint32_t *stream_ring; /* [n_env][624] the env's last 624 twisted MT19937 words (MT's own state,
                              kept one word per draw): required with `stream`; the library
                              writes it before it reads it, no initialisation needed */
    int32_t n_env;
    int32_t state_f64;  /* 0: float arrays, 1: double arrays */
    uint32_t *errors;   /* optional (NULL = not reported): a device word the kernels OR
                           ASTRO_ERR_* bits into when a launch detects an internal fault;
                           the caller clears it and reads it after the launches (the
                           state written by a launch that set a bit is not trusted) */
} AstroState;

/* Bits of AstroState.errors. */
enum {
    ASTRO_ERR_HELPER_WAIT = 1,  /* a helper wave's wait for its step wave's post expired:
                                   that wave's finished games were not re-created */
    ASTRO_ERR_HEADER_WAIT = 2   /* a step wave's wait for its helper's header read expired */
};

/* Control sources of astro_rollout / astro_controls. */
enum {
    ASTRO_POLICY_CONTROL = 0,  /* a control array, int8 [ticks][n_env][nships] */
    ASTRO_POLICY_NOTHING = 1,  /* script.NothingBot (script.py:6-10): every ship 2 */
    ASTRO_POLICY_RANDOM = 2,   /* uniform [0, 6) per ship and tick: splitmix64 of
                                  (global ship id, tick) -- bench.py's `controls` */
    ASTRO_POLICY_BOTS = 3      /* one bot per ship (core.Bots.control, core.py:359-363):
                                  ship s plays bot (bots >> 4s) & 15, an ASTRO_BOT_*,
                                  on its ego view of the state (core.roll_ships) */
};
enum {
    ASTRO_BOT_NOTHING = 0,     /* script.NothingBot */
    ASTRO_BOT_SCRIPT = 1,      /* script.ScriptBot (script.py:13-91): planet avoidance, then
                                  aim at the enemy's forecast; numpy's precision for the
                                  state's dtypes (float32 at a game's first tick) */
    ASTRO_BOT_RANDOM = 2       /* as ASTRO_POLICY_RANDOM for that ship */
};

typedef struct AstroPolicy {
    int32_t kind;          /* ASTRO_POLICY_* */
    int32_t bots;          /* BOTS: ship s's bot = (bots >> (4 * s)) & 15 */
    uint64_t seed;         /* RANDOM */
    int64_t tick0;         /* RANDOM: number of the first tick */
    int64_t env_offset;    /* RANDOM: global id of env 0 (shards) */
    /* ASTRO_BOT_SCRIPT: ScriptBot's constants as the reference evaluates them
       (Python floats; the bot casts them to the state's dtype as numpy does) */
    double script_r2;        /* (planet_radius + ship_radius + avoid_distance) ** 2   script.py:47-49 */
    double script_threshold; /* args['avoid_threshold']                               script.py:71 */
    double ship_thrust;      /* config.ship_thrust                                    script.py:57 */
    double ship_rspeed;      /* config.ship_rspeed                                    script.py:58 */
    double bullet_speed;     /* config.bullet_speed                                   script.py:81 */
    double ship_radius;      /* config.ship_radius                                    script.py:88 */
} AstroPolicy;

/* Statistics accumulated by astro_step when `stats` is non-NULL: uint64
 * [ceil(n_env / 16)][ASTRO_NSTATS], one private row per wave64 (a wave covers
 * 64 envs in the LANE kernel, 16 in the QUAD kernel), added to and never
 * cleared by the library.  Sum the rows for totals.  (A private row per wave keeps the counters contention-free:
 * every wave adding into one shared row serialises at the memory side.) */
enum {
    ASTRO_STAT_BULLETS_IN = 0,  /* live bullets read */
    ASTRO_STAT_BULLETS_OUT = 1, /* live bullets written */
    ASTRO_STAT_RESETS = 2,      /* envs re-created by auto-reset */
    ASTRO_STAT_COLLISIONS = 3,  /* games ended by a ship collision */
    ASTRO_STAT_TIMEOUTS = 4,    /* games ended by max_time */
    ASTRO_STAT_OVERFLOWS = 5,   /* bullets dropped for lack of b_cap */
    ASTRO_STAT_PLANETS = 6,     /* planet slots read */
    ASTRO_STAT_SERIAL = 7,      /* resets the QUAD/PAIR kernels could not make in their
                                   wave-cooperative pass (serial create) */
    ASTRO_NSTATS = 8
};

int astro_abi_version(void);
const char *astro_last_error(void);

/* One tick for every env (core.step).  control: int8 [n_env][nships];
 * reward: float [n_env][nships]; done: uint8 [n_env] (0 running, 1 ship
 * collision, 2 timeout).  Running envs advance in place.  A finished env is
 * re-created from the next seed of its stream when auto_reset != 0 (its
 * state is otherwise undefined until astro_reset). */
int astro_step(const AstroParams *p, const AstroState *s, const int8_t *control,
               float *reward, uint8_t *done, uint64_t *stats, int32_t auto_reset,
               void *stream);

/* k consecutive astro_step calls with controls given up front -- k launches
 * of the one-tick kernel issued from C, arguments checked once: control
 * int8 [k][n_env][nships], reward float [k][n_env][nships], done uint8
 * [k][n_env].  Identical results to k astro_step calls (and to astro_rollout
 * with ASTRO_POLICY_CONTROL, which fuses the k ticks into one launch); for
 * a host loop that has its controls ahead but wants each tick's launch. */
int astro_step_many(const AstroParams *p, const AstroState *s, const int8_t *control, int32_t k,
                    float *reward, uint8_t *done, uint64_t *stats, int32_t auto_reset, void *stream);

/* `ticks` consecutive ticks (each exactly astro_step with auto_reset as
 * given), controls from `policy`: reward float [ticks][n_env][nships], done
 * uint8 [ticks][n_env].  The QUAD kernel runs all ticks in ONE launch, each
 * wave stepping its envs on its own (no grid-wide barrier between ticks);
 * the LANE kernel launches once per tick.  For open-loop control (a policy
 * that needs no observation between ticks). */
int astro_rollout(const AstroParams *p, const AstroState *s, const AstroPolicy *policy, int32_t ticks,
                  const int8_t *control, float *reward, uint8_t *done, uint64_t *stats, int32_t auto_reset,
                  void *stream);

/* core.Bots.control (core.py:359-363) for every env: control int8
 * [n_env][nships] = the controls `policy` picks on the current state (tick
 * policy->tick0 for RANDOM; CONTROL is not a policy here).  The same device
 * code astro_rollout runs each tick, for a host loop that needs the
 * decisions (e.g. to log them) or to check them. */
int astro_controls(const AstroParams *p, const AstroState *s, const AstroPolicy *policy, int8_t *control,
                   void *stream);

/* core.create for the envs with mask[i] != 0 (mask NULL = all): from
 * seeds[i] when seeds != NULL, else from the next seed of env i's stream. */
int astro_reset(const AstroParams *p, const AstroState *s, const uint32_t *seeds,
                const uint8_t *mask, void *stream);

/* Fill table[first .. first+count-1] with key[397] of RandomState(seed)'s
 * init chain (table: uint32 [2^30] for the full range, 4 GiB; ~0.1 s). */
int astro_keytable_build(uint32_t *table, uint32_t first, uint32_t count, void *stream);

/* Position env i's seed stream at generate_configs(seed=stream_seeds[i]) and
 * queue its first game (the next astro_reset without seeds creates it). */
int astro_stream_init(const AstroState *s, const uint32_t *stream_seeds, void *stream);

/* Observation features of every env, as rl.ValueNetwork.get_features then
 * to_batch (rl.py:36-112): out float [n_env][rows][1 + 5*nships + 4]; row r <
 * nplanets is planet r, then the live bullets; column 0 = 0 planet / 1
 * bullet, then every ship's (x, y, dx, dy, norm_angle(b)/pi), then the
 * object's (x, y, dx, dy); rows past the env's objects are -1 (to_batch's
 * padding).  rows = p_pad + b_cap always suffices; objects past `rows` are
 * left out. */
int astro_features(const AstroParams *p, const AstroState *s, float *out, int32_t rows, void *stream);

/* Host memory the kernels can address directly (the single-game path,
 * astro_amd.core: a tick's state lives here, so a step is one launch and one
 * synchronisation, no copies): `bytes` of page-locked, coherent host memory
 * mapped into the device's address space.  *host is the CPU address,
 * *device the address to put in AstroState / pass to the entry points.
 * Every kernel access crosses PCIe: for one or a few games only. */
int astro_host_alloc(uint64_t bytes, void **host, void **device);
int astro_host_free(void *host);

/* One tick of ONE game (core.step, core.py:215-303, as astro/server.py's
 * game_tick and core.play call it), host state in and host state out in a
 * single call: the packed input state is written into the game's arena (host
 * memory the kernel addresses directly, astro_host_alloc), the step kernel
 * runs on `stream`, the call spins until it has finished (hipStreamQuery)
 * and packs the next state.  Packed state layout (float64, the reference
 * State's arrays in order): ships x [S][2], dx [S][2], b [S]; planets x
 * [nplanets][2], dx [nplanets][2]; bullets x [nbullets][2], dx [nbullets][2].
 * Returns 0 (then done / reward / out / out_nbullets are set; out only when
 * done == 0), a negative argument/launch code, or -90 when the launch set
 * AstroState.errors bits (astro_last_error names them). */
typedef struct AstroGameTick {
    AstroParams params;     /* the game's config; the call sets timeout_tick and fire_bits */
    AstroState state;       /* device addresses of the arena's arrays (n_env 1, state_f64 1) */
    void *stream;
    /* host addresses of the same arena bytes */
    int32_t *hdr;
    double *ships, *ships_b, *planets, *bullets;
    int8_t *control;
    uint32_t *fire;
    float *reward;
    uint8_t *done;
    uint32_t *errors;
    /* device addresses of control / fire / reward / done */
    const int8_t *control_dev;
    const uint32_t *fire_dev;
    float *reward_dev;
    uint8_t *done_dev;
    const double *in;       /* host: the input state, packed */
    double *out;            /* host: the next state, packed (room for b_cap bullets) */
    /* this call */
    int32_t nplanets, nbullets;
    int32_t control0, control1;
    int32_t first_step;     /* the game's first step (create()'s float32 arrays: tick 0) */
    int32_t fire_now;       /* reload_time <= reload + dt          core.py:263-267 */
    int32_t timeout_now;    /* max_time <= t + dt                  core.py:257 */
    /* results */
    int32_t out_nbullets;
    int32_t done_out;       /* 0 running, 1 ship collision, 2 timeout */
    float reward_out[2];
    /* completion word in the arena (host and device addresses of one
     * uint32): the tick's wave stores `seq` there after its last store
     * (system-scope release), and the call returns once it reads it, ahead
     * of the stream's own completion; NULL = wait for the stream */
    uint32_t *flag;
    uint32_t *flag_dev;
    uint32_t seq;           /* the call's own counter (astro_game_step increments it) */
    int32_t reserved;
} AstroGameTick;
int astro_game_step(AstroGameTick *t);

/* Device memory of a chosen kind, zeroed, for the per-step state arrays
 * (ships, ships_b, planets, bullets, hdr, reward, done).  A launch reads each
 * of them once and writes each once, so the L2 only holds what the end of
 * the launch must write back:
 *   ASTRO_MEM_DEFAULT     hipMalloc (coarse-grained, cached in L2)
 *   ASTRO_MEM_FINEGRAINED hipDeviceMallocFinegrained
 *   ASTRO_MEM_UNCACHED    hipDeviceMallocUncached (L2 bypassed: stores go
 *                         straight to the memory side, nothing is left
 *                         dirty at the end of a launch)
 * Free with astro_dev_free. */
#define ASTRO_MEM_DEFAULT 0
#define ASTRO_MEM_FINEGRAINED 1
#define ASTRO_MEM_UNCACHED 2
int astro_dev_alloc(uint64_t bytes, int32_t kind, void **device);
int astro_dev_free(void *device);

#ifdef __cplusplus
}
#endif

#endif /* ASTRO_STEP_H */
