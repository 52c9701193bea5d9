/* mjref.h — CPU fp64 oracle for the batched physics step (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * It is the checker, never the product: the product path is libmgx.so (HIP).
 *
 * What it restates: MuJoCo's mj_step pipeline [ext: MuJoCo "Computation" chapter;
 * the reference only calls it, e.g. humanoid_soccer_env/soccer_env.py:414] for the model
 * subset of the seven reference tasks, one function per stage so each HIP stage has a
 * stage-level reference:
 *   mj_checkPos/Vel -> kinematics -> comPos -> crb -> factorM -> collision ->
 *   makeConstraint (limits + pyramidal contacts) -> projectConstraint (A = J M^-1 J' + R) ->
 *   comVel -> passive -> referenceConstraint -> rne -> actuation -> xfrc -> qacc_smooth ->
 *   fwdConstraint (PGS with warmstart) -> checkAcc -> Euler (implicit damping) + integratePos.
 *
 * Parity status: MuJoCo itself is not installed anywhere in this pipeline, so
 * agreement of this oracle with CPU MuJoCo is UNPINNED; it is pinned by known-answer
 * physics tests (tests/test_oracle_physics.py). Env-logic parity is pinned separately by
 * golden vectors generated from the reference's own Python (tests/golden/).
 */
#ifndef MJREF_H_
#define MJREF_H_
#include "../include/mgx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ref_data ref_data;

ref_data *ref_create(const mgx_model_desc *m, int ncon_max, int nefc_max);
void ref_free(ref_data *d);
void ref_reset(const mgx_model_desc *m, ref_data *d);       /* mj_resetData */
void ref_forward(const mgx_model_desc *m, ref_data *d);     /* mj_forward */
void ref_step(const mgx_model_desc *m, ref_data *d);        /* mj_step */
/* test knob: 1 = sum each PGS residual in reverse column order (a different-rounding twin) */
void ref_set_pgs_order(ref_data *d, int reverse);
/* pointer + element count of a named field ("qpos", "xpos", "efc_J", "ncon", ...) */
void *ref_field(ref_data *d, const char *name, int *count);

/* narrowphase test hook: collide geoms g1, g2 of the current geom frames; returns ncon */
int ref_collide_pair(const mgx_model_desc *m, ref_data *d, int pair_index);
/* Newton diagnostics: solves, iterations, active rows over iterations, active-state changes */
void ref_newton_stats(long *out, int reset);
/* narrowphase branch counters since the last reset (16 longs, layout in mjref.c) */
void ref_narrowphase_stats(long *out, int reset);

#ifdef __cplusplus
}
#endif
#endif
