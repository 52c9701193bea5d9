/* mjref.c — CPU fp64 oracle: restatement of MuJoCo's mj_step for the reference tasks.
 * TEST INFRASTRUCTURE ONLY (see mjref.h). Each stage cites the MuJoCo routine it
 * restates [ext] and the reference call site that reaches it.
 */
#include "mjref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define MINVAL 1e-15
#define MAXVAL 1e10
#define MINIMP 0.0001
#define MAXIMP 0.9999
#define MAXCONPAIR 8
#define LS_TOLERANCE 0.01 /* mjOption.ls_tolerance default [ext] */
#define LS_ITERATIONS 50  /* mjOption.ls_iterations default [ext] */

enum { JFREE = 0, JBALL = 1, JSLIDE = 2, JHINGE = 3 };
enum { GPLANE = 0, GHFIELD = 1, GSPHERE = 2, GCAPSULE = 3, GELLIPSOID = 4, GCYLINDER = 5, GBOX = 6 };
enum { C_EQUALITY = 0, C_FRICTION_DOF, C_FRICTION_TENDON, C_LIMIT_JOINT, C_LIMIT_TENDON,
       C_CONTACT_FRICTIONLESS, C_CONTACT_PYRAMIDAL, C_CONTACT_ELLIPTIC };

struct ref_data {
  int ncon_max, nefc_max, nv, nq, nu, nbody, njnt, ngeom, nM;
  /* state */
  double *qpos, *qvel, *qacc_warmstart, *ctrl, *qfrc_applied, *xfrc_applied, *time;
  int *warning;
  /* position stage */
  double *xpos, *xquat, *xmat, *xipos, *ximat, *xanchor, *xaxis, *geom_xpos, *geom_xmat;
  double *subtree_com, *cinert, *cdof, *crb, *qM, *qLD, *qLDiagInv;
  /* velocity / force stage */
  double *cvel, *cdof_dot, *qfrc_bias, *qfrc_passive, *actuator_force, *qfrc_actuator;
  double *qfrc_smooth, *qacc_smooth, *qfrc_constraint, *qacc;
  /* contacts */
  int *ncon;
  double *con_dist, *con_pos, *con_frame, *con_friction, *con_includemargin, *con_solref, *con_solimp;
  int *con_geom, *con_dim, *con_pair;
  /* constraints */
  int *nefc;
  int *efc_type, *efc_id;
  double *efc_J, *efc_pos, *efc_margin, *efc_diagApprox, *efc_R, *efc_D, *efc_KBIP;
  double *efc_vel, *efc_aref, *efc_b, *efc_force, *efc_AR;
  int *solver_niter;
  /* scratch */
  double *scratch;
  /* test knob (ref_set_pgs_order): 1 sums each PGS residual b + sum_c AR_rc f_c in reverse
     column order. The same algorithm with a different fp64 rounding: a twin that measures how
     fast two fp64 implementations of the unconverged 50-sweep solve separate on a trajectory */
  int pgs_reverse;
};

/* ====================================================================== vector helpers */
static double dot3(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void cross3(double *r, const double *a, const double *b) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
static double norm3(const double *a) { return sqrt(dot3(a, a)); }
static double normalize3(double *v) { /* mju_normalize3 */
  double n = norm3(v);
  if (n < MINVAL) { v[0] = 1; v[1] = 0; v[2] = 0; }
  else { double s = 1 / n; v[0] *= s; v[1] *= s; v[2] *= s; }
  return n;
}
static void normalize4(double *q) { /* mju_normalize4 */
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else if (fabs(n - 1) > MINVAL) { double s = 1 / n; q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s; }
}
static void mulquat(double *r, const double *a, const double *b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof t);
}
static void quat2mat(double *r, const double *q) { /* mju_quat2Mat */
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    memcpy(r, I, sizeof I);
    return;
  }
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  r[0] = q00 + q11 - q22 - q33; r[4] = q00 - q11 + q22 - q33; r[8] = q00 - q11 - q22 + q33;
  r[1] = 2 * (q12 - q03); r[2] = 2 * (q13 + q02); r[3] = 2 * (q12 + q03);
  r[5] = 2 * (q23 - q01); r[6] = 2 * (q13 - q02); r[7] = 2 * (q23 + q01);
}
static void rotvecquat(double *r, const double *v, const double *q) { /* mju_rotVecQuat */
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) { r[0] = r[1] = r[2] = 0; return; }
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) { r[0] = v[0]; r[1] = v[1]; r[2] = v[2]; return; }
  double t[3] = {q[0] * v[0] + q[2] * v[2] - q[3] * v[1],
                 q[0] * v[1] + q[3] * v[0] - q[1] * v[2],
                 q[0] * v[2] + q[1] * v[1] - q[2] * v[0]};
  double o[3] = {v[0] + 2 * (q[2] * t[2] - q[3] * t[1]),
                 v[1] + 2 * (q[3] * t[0] - q[1] * t[2]),
                 v[2] + 2 * (q[1] * t[1] - q[2] * t[0])};
  r[0] = o[0]; r[1] = o[1]; r[2] = o[2];
}
static void axisangle2quat(double *q, const double *ax, double ang) {
  if (ang == 0) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  double s = sin(ang * 0.5);
  q[0] = cos(ang * 0.5); q[1] = ax[0] * s; q[2] = ax[1] * s; q[3] = ax[2] * s;
}
static void mulmatvec3(double *r, const double *M, const double *v) { /* r = M v */
  double t[3] = {M[0] * v[0] + M[1] * v[1] + M[2] * v[2], M[3] * v[0] + M[4] * v[1] + M[5] * v[2],
                 M[6] * v[0] + M[7] * v[1] + M[8] * v[2]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
static void mulmatTvec3(double *r, const double *M, const double *v) { /* r = M' v */
  double t[3] = {M[0] * v[0] + M[3] * v[1] + M[6] * v[2], M[1] * v[0] + M[4] * v[1] + M[7] * v[2],
                 M[2] * v[0] + M[5] * v[1] + M[8] * v[2]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
static int isbad(double x) { return x != x || x > MAXVAL || x < -MAXVAL; }
static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* ====================================================================== allocation */
#define ALLOC(f, n) d->f = calloc((size_t)((n) > 0 ? (n) : 1), sizeof(*d->f))

ref_data *ref_create(const mgx_model_desc *m, int ncon_max, int nefc_max) {
  ref_data *d = calloc(1, sizeof(ref_data));
  d->ncon_max = ncon_max; d->nefc_max = nefc_max;
  d->nv = m->nv; d->nq = m->nq; d->nu = m->nu; d->nbody = m->nbody; d->njnt = m->njnt;
  d->ngeom = m->ngeom; d->nM = m->nM;
  int nb = m->nbody, nv = m->nv;
  ALLOC(qpos, m->nq); ALLOC(qvel, nv); ALLOC(qacc_warmstart, nv); ALLOC(ctrl, m->nu);
  ALLOC(qfrc_applied, nv); ALLOC(xfrc_applied, 6 * nb); ALLOC(time, 1); ALLOC(warning, 1);
  ALLOC(xpos, 3 * nb); ALLOC(xquat, 4 * nb); ALLOC(xmat, 9 * nb); ALLOC(xipos, 3 * nb);
  ALLOC(ximat, 9 * nb); ALLOC(xanchor, 3 * m->njnt); ALLOC(xaxis, 3 * m->njnt);
  ALLOC(geom_xpos, 3 * m->ngeom); ALLOC(geom_xmat, 9 * m->ngeom);
  ALLOC(subtree_com, 3 * nb); ALLOC(cinert, 10 * nb); ALLOC(cdof, 6 * nv); ALLOC(crb, 10 * nb);
  ALLOC(qM, m->nM); ALLOC(qLD, m->nM); ALLOC(qLDiagInv, nv);
  ALLOC(cvel, 6 * nb); ALLOC(cdof_dot, 6 * nv); ALLOC(qfrc_bias, nv); ALLOC(qfrc_passive, nv);
  ALLOC(actuator_force, m->nu); ALLOC(qfrc_actuator, nv); ALLOC(qfrc_smooth, nv);
  ALLOC(qacc_smooth, nv); ALLOC(qfrc_constraint, nv); ALLOC(qacc, nv);
  ALLOC(ncon, 1); ALLOC(con_dist, ncon_max); ALLOC(con_pos, 3 * ncon_max);
  ALLOC(con_frame, 9 * ncon_max); ALLOC(con_friction, 5 * ncon_max);
  ALLOC(con_includemargin, ncon_max); ALLOC(con_solref, 2 * ncon_max);
  ALLOC(con_solimp, 5 * ncon_max); ALLOC(con_geom, 2 * ncon_max); ALLOC(con_dim, ncon_max);
  ALLOC(con_pair, ncon_max);
  ALLOC(nefc, 1); ALLOC(efc_type, nefc_max); ALLOC(efc_id, nefc_max);
  ALLOC(efc_J, (size_t)nefc_max * nv); ALLOC(efc_pos, nefc_max); ALLOC(efc_margin, nefc_max);
  ALLOC(efc_diagApprox, nefc_max); ALLOC(efc_R, nefc_max); ALLOC(efc_D, nefc_max);
  ALLOC(efc_KBIP, 4 * nefc_max); ALLOC(efc_vel, nefc_max); ALLOC(efc_aref, nefc_max);
  ALLOC(efc_b, nefc_max); ALLOC(efc_force, nefc_max);
  ALLOC(efc_AR, (size_t)nefc_max * nefc_max); ALLOC(solver_niter, 1);
  ALLOC(scratch, (size_t)nefc_max * nv + 16 * nv + 8 * nefc_max + 64);
  ref_reset(m, d);
  return d;
}

void ref_set_pgs_order(ref_data *d, int reverse) { d->pgs_reverse = reverse != 0; }

void ref_free(ref_data *d) {
  if (!d) return;
  void **p[] = {(void **)&d->qpos, (void **)&d->qvel, (void **)&d->qacc_warmstart, (void **)&d->ctrl,
                (void **)&d->qfrc_applied, (void **)&d->xfrc_applied, (void **)&d->time,
                (void **)&d->warning, (void **)&d->xpos, (void **)&d->xquat, (void **)&d->xmat,
                (void **)&d->xipos, (void **)&d->ximat, (void **)&d->xanchor, (void **)&d->xaxis,
                (void **)&d->geom_xpos, (void **)&d->geom_xmat, (void **)&d->subtree_com,
                (void **)&d->cinert, (void **)&d->cdof, (void **)&d->crb, (void **)&d->qM,
                (void **)&d->qLD, (void **)&d->qLDiagInv, (void **)&d->cvel, (void **)&d->cdof_dot,
                (void **)&d->qfrc_bias, (void **)&d->qfrc_passive, (void **)&d->actuator_force,
                (void **)&d->qfrc_actuator, (void **)&d->qfrc_smooth, (void **)&d->qacc_smooth,
                (void **)&d->qfrc_constraint, (void **)&d->qacc, (void **)&d->ncon,
                (void **)&d->con_dist, (void **)&d->con_pos, (void **)&d->con_frame,
                (void **)&d->con_friction, (void **)&d->con_includemargin, (void **)&d->con_solref,
                (void **)&d->con_solimp, (void **)&d->con_geom, (void **)&d->con_dim,
                (void **)&d->con_pair, (void **)&d->nefc, (void **)&d->efc_type, (void **)&d->efc_id,
                (void **)&d->efc_J, (void **)&d->efc_pos, (void **)&d->efc_margin,
                (void **)&d->efc_diagApprox, (void **)&d->efc_R, (void **)&d->efc_D,
                (void **)&d->efc_KBIP, (void **)&d->efc_vel, (void **)&d->efc_aref, (void **)&d->efc_b,
                (void **)&d->efc_force, (void **)&d->efc_AR, (void **)&d->solver_niter,
                (void **)&d->scratch};
  for (size_t i = 0; i < sizeof p / sizeof p[0]; i++) free(*p[i]);
  free(d);
}

void *ref_field(ref_data *d, const char *name, int *count) {
  struct { const char *n; void *p; int c; } t[] = {
    {"qpos", d->qpos, d->nq}, {"qvel", d->qvel, d->nv}, {"qacc_warmstart", d->qacc_warmstart, d->nv},
    {"ctrl", d->ctrl, d->nu}, {"qfrc_applied", d->qfrc_applied, d->nv},
    {"xfrc_applied", d->xfrc_applied, 6 * d->nbody}, {"time", d->time, 1}, {"warning", d->warning, 1},
    {"xpos", d->xpos, 3 * d->nbody}, {"xquat", d->xquat, 4 * d->nbody}, {"xmat", d->xmat, 9 * d->nbody},
    {"xipos", d->xipos, 3 * d->nbody}, {"ximat", d->ximat, 9 * d->nbody},
    {"xanchor", d->xanchor, 3 * d->njnt}, {"xaxis", d->xaxis, 3 * d->njnt},
    {"geom_xpos", d->geom_xpos, 3 * d->ngeom}, {"geom_xmat", d->geom_xmat, 9 * d->ngeom},
    {"subtree_com", d->subtree_com, 3 * d->nbody}, {"cinert", d->cinert, 10 * d->nbody},
    {"cdof", d->cdof, 6 * d->nv}, {"crb", d->crb, 10 * d->nbody}, {"qM", d->qM, d->nM},
    {"qLD", d->qLD, d->nM}, {"qLDiagInv", d->qLDiagInv, d->nv}, {"cvel", d->cvel, 6 * d->nbody},
    {"cdof_dot", d->cdof_dot, 6 * d->nv}, {"qfrc_bias", d->qfrc_bias, d->nv},
    {"qfrc_passive", d->qfrc_passive, d->nv}, {"actuator_force", d->actuator_force, d->nu},
    {"qfrc_actuator", d->qfrc_actuator, d->nv}, {"qfrc_smooth", d->qfrc_smooth, d->nv},
    {"qacc_smooth", d->qacc_smooth, d->nv}, {"qfrc_constraint", d->qfrc_constraint, d->nv},
    {"qacc", d->qacc, d->nv}, {"ncon", d->ncon, 1}, {"con_dist", d->con_dist, d->ncon_max},
    {"con_pos", d->con_pos, 3 * d->ncon_max}, {"con_frame", d->con_frame, 9 * d->ncon_max},
    {"con_friction", d->con_friction, 5 * d->ncon_max},
    {"con_includemargin", d->con_includemargin, d->ncon_max}, {"con_geom", d->con_geom, 2 * d->ncon_max},
    {"con_dim", d->con_dim, d->ncon_max}, {"con_pair", d->con_pair, d->ncon_max},
    {"nefc", d->nefc, 1}, {"efc_type", d->efc_type, d->nefc_max}, {"efc_id", d->efc_id, d->nefc_max},
    {"efc_J", d->efc_J, d->nefc_max * d->nv}, {"efc_pos", d->efc_pos, d->nefc_max},
    {"efc_margin", d->efc_margin, d->nefc_max}, {"efc_diagApprox", d->efc_diagApprox, d->nefc_max},
    {"efc_R", d->efc_R, d->nefc_max}, {"efc_D", d->efc_D, d->nefc_max},
    {"efc_KBIP", d->efc_KBIP, 4 * d->nefc_max}, {"efc_vel", d->efc_vel, d->nefc_max},
    {"efc_aref", d->efc_aref, d->nefc_max}, {"efc_b", d->efc_b, d->nefc_max},
    {"efc_force", d->efc_force, d->nefc_max}, {"efc_AR", d->efc_AR, d->nefc_max * d->nefc_max},
    {"solver_niter", d->solver_niter, 1},
  };
  for (size_t i = 0; i < sizeof t / sizeof t[0]; i++)
    if (!strcmp(t[i].n, name)) { if (count) *count = t[i].c; return t[i].p; }
  if (count) *count = 0;
  return NULL;
}

/* mj_resetData (engine_io.c) [ext]; reached from soccer_env.py:354 */
void ref_reset(const mgx_model_desc *m, ref_data *d) {
  memcpy(d->qpos, m->qpos0, sizeof(double) * m->nq);
  memset(d->qvel, 0, sizeof(double) * m->nv);
  memset(d->qacc_warmstart, 0, sizeof(double) * m->nv);
  memset(d->ctrl, 0, sizeof(double) * (m->nu > 0 ? m->nu : 1));
  memset(d->qfrc_applied, 0, sizeof(double) * m->nv);
  memset(d->xfrc_applied, 0, sizeof(double) * 6 * m->nbody);
  memset(d->qacc, 0, sizeof(double) * m->nv);
  d->time[0] = 0;
  d->ncon[0] = 0;
  d->nefc[0] = 0;
}

/* ====================================================================== kinematics */
/* mj_kinematics (engine_core_smooth.c) [ext] */
static void kinematics(const mgx_model_desc *m, ref_data *d) {
  d->xpos[0] = d->xpos[1] = d->xpos[2] = 0;
  d->xquat[0] = 1; d->xquat[1] = d->xquat[2] = d->xquat[3] = 0;
  quat2mat(d->xmat, d->xquat);
  for (int i = 1; i < m->nbody; i++) {
    double xpos[3], xquat[4];
    int ja = m->body_jntadr[i], jn = m->body_jntnum[i];
    if (jn == 1 && m->jnt_type[ja] == JFREE) {
      int a = m->jnt_qposadr[ja];
      memcpy(xpos, d->qpos + a, 3 * sizeof(double));
      memcpy(xquat, d->qpos + a + 3, 4 * sizeof(double));
      normalize4(xquat);
      memcpy(d->xanchor + 3 * ja, xpos, 3 * sizeof(double));
      memcpy(d->xaxis + 3 * ja, m->jnt_axis + 3 * ja, 3 * sizeof(double));
    } else {
      int p = m->body_parentid[i];
      mulmatvec3(xpos, d->xmat + 9 * p, m->body_pos + 3 * i);
      for (int k = 0; k < 3; k++) xpos[k] += d->xpos[3 * p + k];
      mulquat(xquat, d->xquat + 4 * p, m->body_quat + 4 * i);
      for (int j = ja; j < ja + jn; j++) {
        int a = m->jnt_qposadr[j];
        rotvecquat(d->xaxis + 3 * j, m->jnt_axis + 3 * j, xquat);
        rotvecquat(d->xanchor + 3 * j, m->jnt_pos + 3 * j, xquat);
        for (int k = 0; k < 3; k++) d->xanchor[3 * j + k] += xpos[k];
        if (m->jnt_type[j] == JSLIDE) {
          double s = d->qpos[a] - m->qpos0[a];
          for (int k = 0; k < 3; k++) xpos[k] += d->xaxis[3 * j + k] * s;
        } else if (m->jnt_type[j] == JHINGE || m->jnt_type[j] == JBALL) {
          double ql[4], v[3];
          if (m->jnt_type[j] == JBALL) { memcpy(ql, d->qpos + a, 4 * sizeof(double)); normalize4(ql); }
          else axisangle2quat(ql, m->jnt_axis + 3 * j, d->qpos[a] - m->qpos0[a]);
          mulquat(xquat, xquat, ql);
          rotvecquat(v, m->jnt_pos + 3 * j, xquat);
          for (int k = 0; k < 3; k++) xpos[k] = d->xanchor[3 * j + k] - v[k];
        }
      }
    }
    normalize4(xquat);
    memcpy(d->xquat + 4 * i, xquat, 4 * sizeof(double));
    memcpy(d->xpos + 3 * i, xpos, 3 * sizeof(double));
    quat2mat(d->xmat + 9 * i, xquat);
  }
  /* inertial frames and geom frames: mj_local2Global */
  for (int i = 0; i < m->nbody; i++) {
    double q[4];
    mulmatvec3(d->xipos + 3 * i, d->xmat + 9 * i, m->body_ipos + 3 * i);
    for (int k = 0; k < 3; k++) d->xipos[3 * i + k] += d->xpos[3 * i + k];
    mulquat(q, d->xquat + 4 * i, m->body_iquat + 4 * i);
    quat2mat(d->ximat + 9 * i, q);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    double q[4];
    mulmatvec3(d->geom_xpos + 3 * g, d->xmat + 9 * b, m->geom_pos + 3 * g);
    for (int k = 0; k < 3; k++) d->geom_xpos[3 * g + k] += d->xpos[3 * b + k];
    mulquat(q, d->xquat + 4 * b, m->geom_quat + 4 * g);
    quat2mat(d->geom_xmat + 9 * g, q);
  }
}

/* mju_dofCom */
static void dofcom(double *res, const double *axis, const double *offset) {
  if (offset) {
    res[0] = axis[0]; res[1] = axis[1]; res[2] = axis[2];
    cross3(res + 3, axis, offset);
  } else {
    res[0] = res[1] = res[2] = 0;
    res[3] = axis[0]; res[4] = axis[1]; res[5] = axis[2];
  }
}

/* mju_inertCom: 10-vector (Ixx Iyy Izz Ixy Ixz Iyz, m*d, m) about the subtree com */
static void inertcom(double *res, const double *inert, const double *mat, const double *dif, double mass) {
  double tmp[9] = {mat[0] * inert[0], mat[3] * inert[0], mat[6] * inert[0],
                   mat[1] * inert[1], mat[4] * inert[1], mat[7] * inert[1],
                   mat[2] * inert[2], mat[5] * inert[2], mat[8] * inert[2]};
  res[0] = mat[0] * tmp[0] + mat[1] * tmp[3] + mat[2] * tmp[6];
  res[1] = mat[3] * tmp[1] + mat[4] * tmp[4] + mat[5] * tmp[7];
  res[2] = mat[6] * tmp[2] + mat[7] * tmp[5] + mat[8] * tmp[8];
  res[3] = mat[0] * tmp[1] + mat[1] * tmp[4] + mat[2] * tmp[7];
  res[4] = mat[0] * tmp[2] + mat[1] * tmp[5] + mat[2] * tmp[8];
  res[5] = mat[3] * tmp[2] + mat[4] * tmp[5] + mat[5] * tmp[8];
  res[0] += mass * (dif[1] * dif[1] + dif[2] * dif[2]);
  res[1] += mass * (dif[0] * dif[0] + dif[2] * dif[2]);
  res[2] += mass * (dif[0] * dif[0] + dif[1] * dif[1]);
  res[3] -= mass * dif[0] * dif[1];
  res[4] -= mass * dif[0] * dif[2];
  res[5] -= mass * dif[1] * dif[2];
  res[6] = mass * dif[0]; res[7] = mass * dif[1]; res[8] = mass * dif[2];
  res[9] = mass;
}

/* mj_comPos [ext] */
static void compos(const mgx_model_desc *m, ref_data *d) {
  double *mass_sub = d->scratch;
  memset(mass_sub, 0, sizeof(double) * m->nbody);
  memset(d->subtree_com, 0, sizeof(double) * 3 * m->nbody);
  for (int i = m->nbody - 1; i >= 0; i--) {
    for (int k = 0; k < 3; k++) d->subtree_com[3 * i + k] += d->xipos[3 * i + k] * m->body_mass[i];
    mass_sub[i] += m->body_mass[i];
    if (i) {
      int p = m->body_parentid[i];
      for (int k = 0; k < 3; k++) d->subtree_com[3 * p + k] += d->subtree_com[3 * i + k];
      mass_sub[p] += mass_sub[i];
    }
    if (mass_sub[i] < MINVAL) memcpy(d->subtree_com + 3 * i, d->xipos + 3 * i, 3 * sizeof(double));
    else for (int k = 0; k < 3; k++) d->subtree_com[3 * i + k] /= (mass_sub[i] > MINVAL ? mass_sub[i] : MINVAL);
  }
  memset(d->cinert, 0, 10 * sizeof(double));
  for (int i = 1; i < m->nbody; i++) {
    double off[3];
    for (int k = 0; k < 3; k++) off[k] = d->xipos[3 * i + k] - d->subtree_com[3 * m->body_rootid[i] + k];
    inertcom(d->cinert + 10 * i, m->body_inertia + 3 * i, d->ximat + 9 * i, off, m->body_mass[i]);
  }
  for (int j = 0; j < m->nv; j++) {
    int b = m->dof_bodyid[j], jid = m->dof_jntid[j];
    double off[3];
    for (int k = 0; k < 3; k++) off[k] = d->subtree_com[3 * m->body_rootid[b] + k] - d->xanchor[3 * jid + k];
    int t = m->jnt_type[jid];
    if (t == JFREE) {
      memset(d->cdof + 6 * j, 0, 18 * sizeof(double));
      for (int k = 0; k < 3; k++) d->cdof[6 * (j + k) + 3 + k] = 1;
      for (int k = 0; k < 3; k++) {
        double ax[3] = {d->xmat[9 * b + k], d->xmat[9 * b + k + 3], d->xmat[9 * b + k + 6]};
        dofcom(d->cdof + 6 * (j + 3 + k), ax, off);
      }
      j += 5;
    } else if (t == JBALL) {
      for (int k = 0; k < 3; k++) {
        double ax[3] = {d->xmat[9 * b + k], d->xmat[9 * b + k + 3], d->xmat[9 * b + k + 6]};
        dofcom(d->cdof + 6 * (j + k), ax, off);
      }
      j += 2;
    } else if (t == JSLIDE) {
      dofcom(d->cdof + 6 * j, d->xaxis + 3 * jid, NULL);
    } else {
      dofcom(d->cdof + 6 * j, d->xaxis + 3 * jid, off);
    }
  }
}

/* mju_mulInertVec: 6D spatial inertia times motion vector */
static void mulinertvec(double *res, const double *i, const double *v) {
  res[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  res[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  res[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  res[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  res[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  res[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
static double dot6(const double *a, const double *b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* mj_crb + dense-forward qM assembly [ext] */
static void crb(const mgx_model_desc *m, ref_data *d) {
  memcpy(d->crb, d->cinert, sizeof(double) * 10 * m->nbody);
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0) for (int k = 0; k < 10; k++) d->crb[10 * p + k] += d->crb[10 * i + k];
  }
  memset(d->qM, 0, sizeof(double) * m->nM);
  for (int i = 0; i < m->nv; i++) {
    double buf[6];
    int adr = m->dof_Madr[i];
    d->qM[adr] = m->dof_armature[i];
    mulinertvec(buf, d->crb + 10 * m->dof_bodyid[i], d->cdof + 6 * i);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) d->qM[adr++] += dot6(d->cdof + 6 * j, buf);
  }
}

/* mj_factorI: M = L' D L, tree-sparse, in place (qLD) [ext] */
static void factor_ld(const mgx_model_desc *m, const double *M, double *LD, double *diaginv) {
  if (LD != M) memcpy(LD, M, sizeof(double) * m->nM);
  for (int k = m->nv - 1; k >= 0; k--) {
    int akk = m->dof_Madr[k];
    if (LD[akk] < MINVAL) LD[akk] = MINVAL;
    int aki = akk + 1;
    int i = m->dof_parentid[k];
    while (i >= 0) {
      double tmp = LD[aki] / LD[akk];
      int cnt = 0;
      for (int j = i; j >= 0; j = m->dof_parentid[j]) cnt++;
      int ai = m->dof_Madr[i];
      for (int s = 0; s < cnt; s++) LD[ai + s] -= LD[aki + s] * tmp;
      LD[aki] = tmp;
      i = m->dof_parentid[i];
      aki++;
    }
  }
  for (int i = 0; i < m->nv; i++) diaginv[i] = 1 / LD[m->dof_Madr[i]];
}

/* mj_solveLD: x = M^-1 x using the L'DL factor */
static void solve_ld(const mgx_model_desc *m, const double *LD, const double *diaginv, double *x) {
  for (int k = m->nv - 1; k >= 0; k--) { /* x <- L'^-1 x */
    double xk = x[k];
    if (xk == 0) continue;
    int a = m->dof_Madr[k] + 1;
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) x[i] -= LD[a++] * xk;
  }
  for (int k = 0; k < m->nv; k++) x[k] *= diaginv[k];
  for (int k = 0; k < m->nv; k++) { /* x <- L^-1 x */
    int a = m->dof_Madr[k] + 1;
    double s = 0;
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) s += LD[a++] * x[i];
    x[k] -= s;
  }
}

/* ====================================================================== jacobians */
static int body_has_dof(const mgx_model_desc *m, int body, int dof) {
  return (m->body_dofmask[body * m->nmaskword + (dof >> 5)] >> (dof & 31)) & 1u;
}
/* mj_jac: translational (jacp, 3 x nv) and rotational (jacr) Jacobians of a point on body */
static void jac(const mgx_model_desc *m, ref_data *d, double *jacp, double *jacr, const double *pt, int body) {
  int nv = m->nv;
  double off[3];
  for (int k = 0; k < 3; k++) off[k] = pt[k] - d->subtree_com[3 * m->body_rootid[body] + k];
  if (jacp) memset(jacp, 0, 3 * nv * sizeof(double));
  if (jacr) memset(jacr, 0, 3 * nv * sizeof(double));
  if (body == 0) return;
  for (int j = 0; j < nv; j++) {
    if (!body_has_dof(m, body, j)) continue;
    const double *c = d->cdof + 6 * j;
    if (jacr) { jacr[j] = c[0]; jacr[j + nv] = c[1]; jacr[j + 2 * nv] = c[2]; }
    if (jacp) {
      double t[3];
      cross3(t, c, off);
      jacp[j] = c[3] + t[0]; jacp[j + nv] = c[4] + t[1]; jacp[j + 2 * nv] = c[5] + t[2];
    }
  }
}

/* ====================================================================== collision */
/* mju_makeFrame: normal -> (normal, tangent1, tangent2) */
static void make_frame(double *f) {
  double tmp[3];
  normalize3(f);
  f[3] = f[4] = f[5] = 0;
  if (f[1] < 0.5 && f[1] > -0.5) f[4] = 1; else f[5] = 1;
  double s = dot3(f, f + 3);
  for (int k = 0; k < 3; k++) tmp[k] = f[k] * s;
  for (int k = 0; k < 3; k++) f[3 + k] -= tmp[k];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

typedef struct { double dist, pos[3], n[3]; } rcon;

static void seg_ends(const double *pos, const double *mat, double hl, double *a, double *b) {
  for (int k = 0; k < 3; k++) { a[k] = pos[k] - hl * mat[3 * k + 2]; b[k] = pos[k] + hl * mat[3 * k + 2]; }
}

/* closest points between segments p1q1 and p2q2 (parameters s, t in [0,1]) */
static void seg_seg(const double *p1, const double *q1, const double *p2, const double *q2, double *s, double *t) {
  double d1[3], d2[3], r[3];
  for (int k = 0; k < 3; k++) { d1[k] = q1[k] - p1[k]; d2[k] = q2[k] - p2[k]; r[k] = p1[k] - p2[k]; }
  double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  if (a <= MINVAL && e <= MINVAL) { *s = *t = 0; return; }
  if (a <= MINVAL) { *s = 0; *t = clampd(f / e, 0, 1); return; }
  double c = dot3(d1, r);
  if (e <= MINVAL) { *t = 0; *s = clampd(-c / a, 0, 1); return; }
  double b = dot3(d1, d2), den = a * e - b * b;
  double ss = den > 1e-12 * a * e ? clampd((b * f - c * e) / den, 0, 1) : 0;
  double tt = (b * ss + f) / e;
  if (tt < 0) { tt = 0; ss = clampd(-c / a, 0, 1); }
  else if (tt > 1) { tt = 1; ss = clampd((b - c) / a, 0, 1); }
  *s = ss; *t = tt;
}

/* signed distance of a box-local point to the box; e = outward unit normal at the closest
 * surface feature (box frame). Inside: nearest face, ties (within 1e-12 of the size) -> lowest axis. */
static double box_sd(const double *p, const double *h, double *e) {
  /* a coordinate within `tie` outside its face plane counts as on it (points placed on a face
     boundary by construction classify the same under any rounding) */
  const double tie = 1e-12 * (h[0] + h[1] + h[2]);
  int outside = 0;
  double q[3], dv[3];
  for (int k = 0; k < 3; k++) {
    q[k] = clampd(p[k], -h[k], h[k]);
    dv[k] = p[k] - q[k];
    if (fabs(dv[k]) <= tie) dv[k] = 0;
    if (dv[k] != 0) outside = 1;
  }
  if (outside) {
    double L = normalize3(dv);
    e[0] = dv[0]; e[1] = dv[1]; e[2] = dv[2];
    return L;
  }
  /* faces within `tie` of the nearest count as equally near: the lowest axis wins (a capsule
     axis's deepest point inside a box sits where two face distances are equal) */
  int best = 0;
  double bd = h[0] - fabs(p[0]);
  for (int k = 1; k < 3; k++) {
    double dk = h[k] - fabs(p[k]);
    if (dk < bd - tie) { bd = dk; best = k; }
  }
  e[0] = e[1] = e[2] = 0;
  e[best] = p[best] >= -tie ? 1 : -1; /* on the mid-plane (within tie) the + face */
  return -bd;
}

/* sphere (center c world, radius r) vs box geom; normal from sphere to box */
static int sphere_box_core(const double *c, double r, const double *bp, const double *bm, const double *h,
                           double margin, rcon *out) {
  double tmp[3] = {c[0] - bp[0], c[1] - bp[1], c[2] - bp[2]}, pl[3], e[3], ew[3];
  mulmatTvec3(pl, bm, tmp);
  double sd = box_sd(pl, h, e);
  double dist = sd - r;
  if (dist > margin) return 0;
  mulmatvec3(ew, bm, e);
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = -ew[k]; out->pos[k] = c[k] - ew[k] * (r + 0.5 * dist); }
  return 1;
}

/* Narrowphase branch counters (test infrastructure: tools/narrowphase_stats.py reads them at
 * bench conditions): [0] capsule-box pairs with 1 contact, [1] with 2, [2] capsule-capsule
 * general, [3] capsule-capsule parallel branch, [4] its contacts, [5..13] box-box pairs by
 * contact count 0..8 */
static long g_np_stats[16];
void ref_narrowphase_stats(long *out, int reset) {
  for (int k = 0; k < 16; k++) out[k] = g_np_stats[k];
  if (reset) memset(g_np_stats, 0, sizeof(g_np_stats));
}

/* point of a capsule axis c + s a (box frame, s in [-1, 1]) closest to / deepest in the box:
 * the convex signed distance d(s) is minimised over its ends, kinks (face-plane and zero
 * crossings, equal inside face distances) and the stationary points of its outside pieces (26
 * sign patterns); the lowest s within tol of the minimum wins (mgx_collide.h capsule_box_segpos) */
static double capsule_box_segpos(const double *c, const double *a, const double *h) {
  double best = 1e30, e[3], p[3], cand[49], dv[49];
  double hm = h[0] > h[1] ? (h[0] > h[2] ? h[0] : h[2]) : (h[1] > h[2] ? h[1] : h[2]);
  const double tol = 1e-10 * (1 + hm);
  int nc = 0;
  cand[nc++] = -1;
  cand[nc++] = 1;
  for (int i = 0; i < 3; i++)
    if (fabs(a[i]) > MINVAL) {
      cand[nc++] = (h[i] - c[i]) / a[i];
      cand[nc++] = (-h[i] - c[i]) / a[i];
      cand[nc++] = -c[i] / a[i];
    }
  for (int i = 0; i < 3; i++)
    for (int j = i + 1; j < 3; j++)
      for (int sg = 0; sg < 4; sg++) {
        double si = (sg & 1) ? -1 : 1, sj = (sg & 2) ? -1 : 1;
        double den = sj * a[j] - si * a[i];
        if (fabs(den) > MINVAL) cand[nc++] = (h[j] - h[i] - sj * c[j] + si * c[i]) / den;
      }
  for (int pat = 1; pat < 27; pat++) {
    double num = 0, den = 0;
    int q = pat;
    for (int i = 0; i < 3; i++, q /= 3) {
      int st = q % 3;
      if (!st) continue;
      double sg = st == 1 ? 1 : -1;
      num += a[i] * (sg * h[i] - c[i]);
      den += a[i] * a[i];
    }
    if (den > MINVAL) cand[nc++] = num / den;
  }
  for (int k = 0; k < nc; k++) {
    double sk = clampd(cand[k], -1, 1);
    cand[k] = sk;
    for (int i = 0; i < 3; i++) p[i] = c[i] + sk * a[i];
    dv[k] = box_sd(p, h, e);
    if (dv[k] < best) best = dv[k];
  }
  double bs = 2;
  for (int k = 0; k < nc; k++)
    if (dv[k] <= best + tol && cand[k] < bs) bs = cand[k];
  return bs;
}

/* sphere of radius r at box-frame point pl (world point w) vs the box */
static int sphere_box_local(const double *pl, const double *w, double r, const double *bm, const double *h,
                            double margin, double *e, rcon *out) {
  double sd = box_sd(pl, h, e), dist = sd - r, ew[3];
  if (dist > margin) return 0;
  mulmatvec3(ew, bm, e);
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = -ew[k]; out->pos[k] = w[k] - ew[k] * (r + 0.5 * dist); }
  return 1;
}

/* capsule (geom1) vs box (geom2), <= 2 contacts, structured as mjc_CapsuleBox [ext]: the axis
 * point closest to / deepest in the box as a sphere-box contact; when it is on a box face, a
 * second sphere-box contact at the far end of the axis's overlap with the face rectangle if
 * that point is within margin of the same face (dropped within a tenth of the radius of the
 * first). The thresholds are this restatement's: MuJoCo's source is not available here. */
static int capsule_box(const double *cp, const double *cm, const double *cs, const double *bp, const double *bm,
                       const double *h, double margin, rcon *out) {
  double r = cs[0], hl = cs[1];
  double tmp[3] = {cp[0] - bp[0], cp[1] - bp[1], cp[2] - bp[2]}, c[3], a[3];
  double ax[3] = {cm[2] * hl, cm[5] * hl, cm[8] * hl};
  mulmatTvec3(c, bm, tmp);
  mulmatTvec3(a, bm, ax);
  double s1 = capsule_box_segpos(c, a, h), pl[3], w[3], e[3], e2[3];
  for (int k = 0; k < 3; k++) { pl[k] = c[k] + s1 * a[k]; w[k] = cp[k] + s1 * ax[k]; }
  if (!sphere_box_local(pl, w, r, bm, h, margin, e, out)) return 0;
  int fk = -1, nz = 0, n = 1;
  for (int k = 0; k < 3; k++)
    if (e[k] != 0) { nz++; fk = k; }
  double lo = -1, hi = 1;
  int ok = nz == 1;
  for (int i = 0; i < 3 && ok; i++) {
    if (i == fk) continue;
    if (fabs(a[i]) > MINVAL) {
      double t0 = (-h[i] - c[i]) / a[i], t1 = (h[i] - c[i]) / a[i];
      if (t0 > t1) { double t = t0; t0 = t1; t1 = t; }
      lo = t0 > lo ? t0 : lo;
      hi = t1 < hi ? t1 : hi;
    } else if (fabs(c[i]) > h[i]) {
      ok = 0;
    }
  }
  if (ok && lo <= hi) {
    double s2 = (s1 - lo < hi - s1) ? hi : lo;
    if (fabs(s2 - s1) * hl >= 0.1 * r) {
      for (int k = 0; k < 3; k++) { pl[k] = c[k] + s2 * a[k]; w[k] = cp[k] + s2 * ax[k]; }
      /* the far point must lie on the same face: one nonzero normal component, same axis and sign */
      if (sphere_box_local(pl, w, r, bm, h, margin, e2, out + 1) && (e2[0] != 0) + (e2[1] != 0) + (e2[2] != 0) == 1 &&
          e2[fk] * e[fk] > 0)
        n = 2;
    }
  }
  g_np_stats[n - 1]++;
  return n;
}

/* mjraw_SphereSphere [ext]: coincident centres take the cross product of the geoms' z axes */
static int sph_sph_raw(const double *c1, const double *m1, double r1, const double *c2, const double *m2, double r2,
                       double margin, rcon *out) {
  double dv[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
  double dist = sqrt(dot3(dv, dv)) - r1 - r2;
  if (dist > margin) return 0;
  double L = normalize3(dv);
  if (L < MINVAL) {
    double z1[3] = {m1[2], m1[5], m1[8]}, z2[3] = {m2[2], m2[5], m2[8]};
    cross3(dv, z1, z2);
    normalize3(dv);
  }
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = dv[k]; out->pos[k] = c1[k] + dv[k] * (r1 + 0.5 * dist); }
  return 1;
}

/* mjc_CapsuleCapsule [ext]: centre + half-axis form, MuJoCo's clamping sequence; parallel axes
 * (|det| < mjMINVAL): axis ends x1 = +-1 then x2 = +-1, stopping at two contacts */
static int capsule_capsule(const double *p1, const double *m1, const double *s1, const double *p2, const double *m2,
                           const double *s2, double margin, rcon *out) {
  double a1[3] = {m1[2] * s1[1], m1[5] * s1[1], m1[8] * s1[1]};
  double a2[3] = {m2[2] * s2[1], m2[5] * s2[1], m2[8] * s2[1]};
  double dif[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  double ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
  double u = -dot3(a1, dif), v = dot3(a2, dif);
  double det = ma * mc - mb * mb, v1[3], v2[3];
  if (fabs(det) >= MINVAL) {
    double x1 = (mc * u - mb * v) / det, x2 = (ma * v - mb * u) / det;
    if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
    else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
    if (x2 > 1) { x2 = 1; x1 = clampd((u - mb) / ma, -1, 1); }
    else if (x2 < -1) { x2 = -1; x1 = clampd((u + mb) / ma, -1, 1); }
    for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + a2[k] * x2; }
    g_np_stats[2]++;
    return sph_sph_raw(v1, m1, s1[0], v2, m2, s2[0], margin, out);
  }
  int n = 0;
  for (int e = 0; e < 4 && n < 2; e++) {
    double sg = (e & 1) ? -1 : 1;
    if (e < 2) {
      double x2 = clampd((v - sg * mb) / mc, -1, 1);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + sg * a1[k]; v2[k] = p2[k] + a2[k] * x2; }
    } else {
      double x1 = clampd((u - sg * mb) / ma, -1, 1);
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + a1[k] * x1; v2[k] = p2[k] + sg * a2[k]; }
    }
    n += sph_sph_raw(v1, m1, s1[0], v2, m2, s2[0], margin, out + n);
  }
  g_np_stats[3]++;
  g_np_stats[4] += n;
  return n;
}

/* mjc_SphereCapsule [ext]: the sphere centre projected on the axis, clamped to the half-length */
static int sphere_capsule(const double *p1, const double *m1, const double *s1, const double *p2, const double *m2,
                          const double *s2, double margin, rcon *out) {
  double ax[3] = {m2[2], m2[5], m2[8]}, dv[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
  double x = clampd(dot3(ax, dv), -s2[1], s2[1]);
  double q[3] = {p2[0] + ax[0] * x, p2[1] + ax[1] * x, p2[2] + ax[2] * x};
  return sph_sph_raw(p1, m1, s1[0], q, m2, s2[0], margin, out);
}

/* ---- cylinders (bipedal_rescue: sphere/capsule/box vs static cylinders) [ext]
 * MuJoCo routes these pairs through its general convex collider (one contact per pair);
 * this restatement keeps the one-contact semantics with closed forms on the exact
 * cylinder signed distance, which is convex, so 1-D searches along segments are exact. */

/* signed distance of a cylinder-local point (radius r, half-height hh, axis z);
 * e = outward unit normal of the closest surface feature (cylinder frame) */
static double cyl_sd(const double *p, double r, double hh, double *e) {
  double rho = sqrt(p[0] * p[0] + p[1] * p[1]);
  double dr = rho - r, dz = fabs(p[2]) - hh;
  double ux = 1, uy = 0, sz = p[2] >= 0 ? 1 : -1;
  if (rho > MINVAL) { ux = p[0] / rho; uy = p[1] / rho; }
  if (dr > 0 && dz > 0) { /* rim region */
    double L = sqrt(dr * dr + dz * dz);
    e[0] = ux * dr / L; e[1] = uy * dr / L; e[2] = sz * dz / L;
    return L;
  }
  if (dr >= dz) { e[0] = ux; e[1] = uy; e[2] = 0; return dr; }
  e[0] = 0; e[1] = 0; e[2] = sz;
  return dz;
}

/* sphere (center c world, radius R) vs cylinder geom; normal from sphere to cylinder */
static int sphere_cyl_core(const double *c, double R, const double *yp, const double *ym, const double *ys,
                           double margin, rcon *out) {
  double tmp[3] = {c[0] - yp[0], c[1] - yp[1], c[2] - yp[2]}, pl[3], e[3], ew[3];
  mulmatTvec3(pl, ym, tmp);
  double dist = cyl_sd(pl, ys[0], ys[1], e) - R;
  if (dist > margin) return 0;
  mulmatvec3(ew, ym, e);
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = -ew[k]; out->pos[k] = c[k] - ew[k] * (R + 0.5 * dist); }
  return 1;
}

/* capsule (geom1) vs cylinder (geom2): the deepest point of the capsule segment (golden
 * section over the convex profile, or an endpoint) as a sphere-cylinder contact */
static int capsule_cyl(const double *cp, const double *cm, const double *cs, const double *yp, const double *ym,
                       const double *ys, double margin, rcon *out) {
  double a[3], b[3], al[3], bl[3], tmp[3], e[3], p[3];
  seg_ends(cp, cm, cs[1], a, b);
  for (int k = 0; k < 3; k++) tmp[k] = a[k] - yp[k];
  mulmatTvec3(al, ym, tmp);
  for (int k = 0; k < 3; k++) tmp[k] = b[k] - yp[k];
  mulmatTvec3(bl, ym, tmp);
  double lo = 0, hi = 1;
  const double gr = 0.6180339887498949;
  double x1 = hi - gr * (hi - lo), x2 = lo + gr * (hi - lo), f1, f2;
  for (int k = 0; k < 3; k++) p[k] = al[k] + x1 * (bl[k] - al[k]);
  f1 = cyl_sd(p, ys[0], ys[1], e);
  for (int k = 0; k < 3; k++) p[k] = al[k] + x2 * (bl[k] - al[k]);
  f2 = cyl_sd(p, ys[0], ys[1], e);
  for (int it = 0; it < 40; it++) {
    if (f1 <= f2) {
      hi = x2; x2 = x1; f2 = f1; x1 = hi - gr * (hi - lo);
      for (int k = 0; k < 3; k++) p[k] = al[k] + x1 * (bl[k] - al[k]);
      f1 = cyl_sd(p, ys[0], ys[1], e);
    } else {
      lo = x1; x1 = x2; f1 = f2; x2 = lo + gr * (hi - lo);
      for (int k = 0; k < 3; k++) p[k] = al[k] + x2 * (bl[k] - al[k]);
      f2 = cyl_sd(p, ys[0], ys[1], e);
    }
  }
  double ts = 0.5 * (lo + hi);
  for (int k = 0; k < 3; k++) p[k] = al[k] + ts * (bl[k] - al[k]);
  double fs = cyl_sd(p, ys[0], ys[1], e), f0 = cyl_sd(al, ys[0], ys[1], e), fb = cyl_sd(bl, ys[0], ys[1], e);
  double t = ts;
  if (f0 <= fs && f0 <= fb) t = 0;
  else if (fb < fs) t = 1;
  double cw[3];
  for (int k = 0; k < 3; k++) cw[k] = a[k] + t * (b[k] - a[k]);
  return sphere_cyl_core(cw, cs[0], yp, ym, ys, margin, out);
}

/* cylinder (geom1) vs box (geom2): the deeper of (a) the box vertex deepest in the
 * cylinder and (b) the cylinder support point deepest in the box, found by 3 fixed-point
 * steps d <- -(box normal at the current point); one contact, normal from cylinder to box */
static int cyl_box(const double *yp, const double *ym, const double *ys, const double *bp, const double *bm,
                   const double *h, double margin, rcon *out) {
  double best = 1e300, bn[3] = {0, 0, 1}, bpos[3] = {0, 0, 0};
  double v[3], w[3], tmp[3], pl[3], e[3], ew[3];
  for (int i = 0; i < 8; i++) {
    v[0] = (i & 1) ? h[0] : -h[0]; v[1] = (i & 2) ? h[1] : -h[1]; v[2] = (i & 4) ? h[2] : -h[2];
    mulmatvec3(w, bm, v);
    for (int k = 0; k < 3; k++) { w[k] += bp[k]; tmp[k] = w[k] - yp[k]; }
    mulmatTvec3(pl, ym, tmp);
    double sd = cyl_sd(pl, ys[0], ys[1], e);
    if (sd < best) {
      best = sd;
      mulmatvec3(ew, ym, e);
      for (int k = 0; k < 3; k++) { bn[k] = ew[k]; bpos[k] = w[k] - 0.5 * sd * ew[k]; }
    }
  }
  double q[3] = {yp[0], yp[1], yp[2]};
  for (int it = 0; it < 3; it++) {
    for (int k = 0; k < 3; k++) tmp[k] = q[k] - bp[k];
    mulmatTvec3(pl, bm, tmp);
    box_sd(pl, h, e);
    double d[3], dl[3];
    mulmatvec3(ew, bm, e);
    for (int k = 0; k < 3; k++) d[k] = -ew[k];
    mulmatTvec3(dl, ym, d);
    double rxy = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
    double sl[3] = {0, 0, dl[2] >= 0 ? ys[1] : -ys[1]};
    if (rxy > MINVAL) { sl[0] = ys[0] * dl[0] / rxy; sl[1] = ys[0] * dl[1] / rxy; }
    mulmatvec3(q, ym, sl);
    for (int k = 0; k < 3; k++) q[k] += yp[k];
    for (int k = 0; k < 3; k++) tmp[k] = q[k] - bp[k];
    mulmatTvec3(pl, bm, tmp);
    double sd = box_sd(pl, h, e);
    if (sd < best) {
      best = sd;
      mulmatvec3(ew, bm, e);
      for (int k = 0; k < 3; k++) { bn[k] = -ew[k]; bpos[k] = q[k] - 0.5 * sd * ew[k]; }
    }
  }
  if (best > margin) return 0;
  out->dist = best;
  for (int k = 0; k < 3; k++) { out->n[k] = bn[k]; out->pos[k] = bpos[k]; }
  return 1;
}

/* cylinder support point (world) in world direction d: the rim point on the side d leans to,
 * the face centre when d is along the axis */
static void cyl_support(const double *yp, const double *ym, const double *ys, const double *d, double *q) {
  double dl[3];
  mulmatTvec3(dl, ym, d);
  double rxy = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
  double sl[3] = {0, 0, dl[2] >= 0 ? ys[1] : -ys[1]};
  if (rxy > MINVAL) { sl[0] = ys[0] * dl[0] / rxy; sl[1] = ys[0] * dl[1] / rxy; }
  mulmatvec3(q, ym, sl);
  for (int k = 0; k < 3; k++) q[k] += yp[k];
}

/* signed distance of world point w to a cylinder geom; e = outward normal (world) */
static double cyl_sd_world(const double *yp, const double *ym, const double *ys, const double *w, double *ew) {
  double tmp[3] = {w[0] - yp[0], w[1] - yp[1], w[2] - yp[2]}, pl[3], e[3];
  mulmatTvec3(pl, ym, tmp);
  double sd = cyl_sd(pl, ys[0], ys[1], e);
  mulmatvec3(ew, ym, e);
  return sd;
}

/* cylinder (geom1) vs cylinder (geom2) [ext]: MuJoCo routes this pair through its general
 * convex collider (one contact). Own restatement with the same one-contact semantics, built
 * like cyl_box's support search: (a) the point of cylinder 2 deepest in cylinder 1, found by 4
 * fixed-point steps q <- support_2(-n_1(q)) from cylinder 2's centre, normal = n_1 (out of 1);
 * (b) the same with the roles swapped, normal = -n_2; the deeper candidate wins. The contact
 * point sits half the depth back along the normal. */
static int cyl_cyl(const double *ap, const double *am, const double *as, const double *bp, const double *bm,
                   const double *bs, double margin, rcon *out) {
  double best = 1e300, bn[3] = {0, 0, 1}, bpos[3] = {0, 0, 0};
  for (int side = 0; side < 2; side++) {
    /* side 0: points of B in A; side 1: points of A in B */
    const double *fp = side ? bp : ap, *fm = side ? bm : am, *fs = side ? bs : as;  /* the SDF body */
    const double *sp = side ? ap : bp, *sm = side ? am : bm, *ss = side ? as : bs;  /* the support body */
    double q[3] = {sp[0], sp[1], sp[2]}, ew[3], d[3];
    for (int it = 0; it < 4; it++) {
      cyl_sd_world(fp, fm, fs, q, ew);
      for (int k = 0; k < 3; k++) d[k] = -ew[k];
      cyl_support(sp, sm, ss, d, q);
      double sd = cyl_sd_world(fp, fm, fs, q, ew);
      if (sd < best) {
        best = sd;
        for (int k = 0; k < 3; k++) {
          bn[k] = side ? -ew[k] : ew[k];
          bpos[k] = q[k] - 0.5 * sd * ew[k];
        }
      }
    }
  }
  if (best > margin) return 0;
  out->dist = best;
  for (int k = 0; k < 3; k++) { out->n[k] = bn[k]; out->pos[k] = bpos[k]; }
  return 1;
}

/* box (geom1) vs box (geom2): separating-axis test over 15 axes, then face clipping
 * (reference face vs incident face, up to 8 points) or one edge-edge contact. */
static int clip_poly(double (*in)[2], int n, int axis, double lim, double sgn, double tol, double (*out)[2]) {
  int m = 0;
  for (int i = 0; i < n; i++) {
    double *P = in[i], *Q = in[(i + 1) % n];
    double dp = sgn * P[axis] - lim, dq = sgn * Q[axis] - lim;
    if (dp <= tol && m < 8) { out[m][0] = P[0]; out[m][1] = P[1]; m++; }
    if (m < 8 && ((dp < -tol && dq > tol) || (dp > tol && dq < -tol))) {
      double t = dp / (dp - dq);
      out[m][0] = P[0] + t * (Q[0] - P[0]);
      out[m][1] = P[1] + t * (Q[1] - P[1]);
      m++;
    }
  }
  return m;
}

static int box_box(const double *pa, const double *Ra, const double *ha, const double *pb, const double *Rb,
                   const double *hb, double margin, rcon *out) {
  double d[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  double A[3][3], B[3][3]; /* A[i] = i-th axis of box a (column i of Ra) */
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { A[i][k] = Ra[3 * k + i]; B[i][k] = Rb[3 * k + i]; }
  double best_face = -1e30, best_edge = -1e30;
  int face_axis = -1, edge_i = -1, edge_j = -1;
  /* face axes within ftol of the best keep the earlier one (box a before box b): equal
   * separations of aligned boxes then pick the same reference face whatever the rounding */
  double hmax = 0;
  for (int k = 0; k < 3; k++) { hmax = ha[k] > hmax ? ha[k] : hmax; hmax = hb[k] > hmax ? hb[k] : hmax; }
  const double ftol = 1e-6 * hmax;
  double edge_n[3] = {0, 0, 0};
  for (int ax = 0; ax < 6; ax++) {
    const double *n = ax < 3 ? A[ax] : B[ax - 3];
    double ra = 0, rb = 0;
    for (int k = 0; k < 3; k++) { ra += ha[k] * fabs(dot3(A[k], n)); rb += hb[k] * fabs(dot3(B[k], n)); }
    double s = fabs(dot3(d, n)) - ra - rb;
    if (s > margin) return 0;
    if (s > best_face + ftol) { best_face = s; face_axis = ax; }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double n[3];
      cross3(n, A[i], B[j]);
      double L = norm3(n);
      if (L < 1e-6) continue;
      for (int k = 0; k < 3; k++) n[k] /= L;
      double ra = 0, rb = 0;
      for (int k = 0; k < 3; k++) { ra += ha[k] * fabs(dot3(A[k], n)); rb += hb[k] * fabs(dot3(B[k], n)); }
      double s = fabs(dot3(d, n)) - ra - rb;
      if (s > margin) return 0;
      if (s > best_edge) { best_edge = s; edge_i = i; edge_j = j; memcpy(edge_n, n, sizeof edge_n); }
    }
  if (edge_i >= 0 && best_edge > best_face + 1e-5 + 0.05 * fabs(best_face)) {
    double n[3] = {edge_n[0], edge_n[1], edge_n[2]};
    if (dot3(n, d) < 0) for (int k = 0; k < 3; k++) n[k] = -n[k];
    double ca[3], cb[3];
    memcpy(ca, pa, sizeof ca);
    memcpy(cb, pb, sizeof cb);
    for (int k = 0; k < 3; k++) {
      if (k != edge_i) { double sg = dot3(A[k], n) >= 0 ? 1 : -1; for (int c = 0; c < 3; c++) ca[c] += sg * ha[k] * A[k][c]; }
      if (k != edge_j) { double sg = dot3(B[k], n) <= 0 ? 1 : -1; for (int c = 0; c < 3; c++) cb[c] += sg * hb[k] * B[k][c]; }
    }
    double a0[3], a1[3], b0[3], b1[3], s, t, P[3], Q[3];
    for (int c = 0; c < 3; c++) {
      a0[c] = ca[c] - ha[edge_i] * A[edge_i][c]; a1[c] = ca[c] + ha[edge_i] * A[edge_i][c];
      b0[c] = cb[c] - hb[edge_j] * B[edge_j][c]; b1[c] = cb[c] + hb[edge_j] * B[edge_j][c];
    }
    seg_seg(a0, a1, b0, b1, &s, &t);
    for (int c = 0; c < 3; c++) { P[c] = a0[c] + s * (a1[c] - a0[c]); Q[c] = b0[c] + t * (b1[c] - b0[c]); }
    double dq[3] = {Q[0] - P[0], Q[1] - P[1], Q[2] - P[2]};
    out[0].dist = dot3(dq, n);
    if (out[0].dist > margin) return 0;
    for (int c = 0; c < 3; c++) { out[0].n[c] = n[c]; out[0].pos[c] = 0.5 * (P[c] + Q[c]); }
    return 1;
  }
  /* a NaN pose fails every separation test and leaves no axis selected: no contact (indexing
     with face_axis = -1 would read before the size and axis arrays) */
  if (face_axis < 0) return 0;
  /* face contact: reference box R, incident box I */
  int refA = face_axis < 3;
  int ri = refA ? face_axis : face_axis - 3;
  const double *pr = refA ? pa : pb, *pi = refA ? pb : pa;
  const double *hr = refA ? ha : hb, *hi = refA ? hb : ha;
  double (*R)[3] = refA ? A : B, (*I)[3] = refA ? B : A;
  double toI[3] = {pi[0] - pr[0], pi[1] - pr[1], pi[2] - pr[2]};
  double nr[3];
  double sg = dot3(toI, R[ri]) >= 0 ? 1 : -1;
  for (int k = 0; k < 3; k++) nr[k] = sg * R[ri][k];
  /* incident face: most anti-parallel to nr */
  int ii = 0;
  double bestd = -1;
  for (int k = 0; k < 3; k++) { double v = fabs(dot3(I[k], nr)); if (v > bestd) { bestd = v; ii = k; } }
  double si = dot3(I[ii], nr) > 0 ? -1 : 1;
  double fc[3];
  for (int k = 0; k < 3; k++) fc[k] = pi[k] + si * hi[ii] * I[ii][k];
  int u = (ii + 1) % 3, v = (ii + 2) % 3;
  int ru = (ri + 1) % 3, rv = (ri + 2) % 3;
  double poly[8][2], tmp[8][2];
  const double sgn4[4][2] = {{1, 1}, {-1, 1}, {-1, -1}, {1, -1}};
  for (int c = 0; c < 4; c++) {
    double P[3], rel[3];
    for (int k = 0; k < 3; k++)
      P[k] = fc[k] + sgn4[c][0] * hi[u] * I[u][k] + sgn4[c][1] * hi[v] * I[v][k];
    for (int k = 0; k < 3; k++) rel[k] = P[k] - pr[k];
    poly[c][0] = dot3(rel, R[ru]);
    poly[c][1] = dot3(rel, R[rv]);
  }
  /* vertices within tol of a clip line count as on it (inside, no intersection point): aligned
   * faces of equal extent (the gripper fingers) then clip to the same polygon whatever the
   * rounding of the coordinates */
  const double tol = 1e-5 * (hr[ru] > hr[rv] ? hr[ru] : hr[rv]);
  int np = 4;
  np = clip_poly(poly, np, 0, hr[ru], 1, tol, tmp);
  np = clip_poly(tmp, np, 0, hr[ru], -1, tol, poly);
  np = clip_poly(poly, np, 1, hr[rv], 1, tol, tmp);
  np = clip_poly(tmp, np, 1, hr[rv], -1, tol, poly);
  /* depth of each clipped point: intersect the incident face plane along nr */
  double fn[3];
  for (int k = 0; k < 3; k++) fn[k] = si * I[ii][k];
  double fndn = dot3(fn, nr);
  int n = 0;
  for (int c = 0; c < np && n < MAXCONPAIR; c++) {
    double P[3];
    for (int k = 0; k < 3; k++) P[k] = pr[k] + poly[c][0] * R[ru][k] + poly[c][1] * R[rv][k] + hr[ri] * nr[k];
    /* move P along nr onto the incident face plane: (P + t nr - fc).fn = 0 */
    double rel[3] = {P[0] - fc[0], P[1] - fc[1], P[2] - fc[2]};
    double t = fabs(fndn) > MINVAL ? -dot3(rel, fn) / fndn : 0;
    double depth = t; /* signed distance from reference face to incident point along nr */
    if (depth > margin) continue;
    out[n].dist = depth;
    for (int k = 0; k < 3; k++) {
      out[n].n[k] = refA ? nr[k] : -nr[k];
      out[n].pos[k] = P[k] + 0.5 * t * nr[k];
    }
    n++;
  }
  return n;
}

/* plane (geom1, infinite, normal = local z) vs primitives */
static int plane_sphere(const double *pp, const double *pm, const double *c, double r, double margin, rcon *out) {
  double n[3] = {pm[2], pm[5], pm[8]};
  double rel[3] = {c[0] - pp[0], c[1] - pp[1], c[2] - pp[2]};
  double dist = dot3(rel, n) - r;
  if (dist > margin) return 0;
  out->dist = dist;
  for (int k = 0; k < 3; k++) { out->n[k] = n[k]; out->pos[k] = c[k] - n[k] * (r + 0.5 * dist); }
  return 1;
}

static int plane_box(const double *pp, const double *pm, const double *bp, const double *bm, const double *h,
                     double margin, rcon *out) {
  double n[3] = {pm[2], pm[5], pm[8]};
  int cnt = 0;
  for (int c = 0; c < 8 && cnt < 4; c++) {
    double v[3], loc[3] = {(c & 1) ? h[0] : -h[0], (c & 2) ? h[1] : -h[1], (c & 4) ? h[2] : -h[2]};
    mulmatvec3(v, bm, loc);
    for (int k = 0; k < 3; k++) v[k] += bp[k];
    double rel[3] = {v[0] - pp[0], v[1] - pp[1], v[2] - pp[2]};
    double dist = dot3(rel, n);
    if (dist > margin) continue;
    out[cnt].dist = dist;
    for (int k = 0; k < 3; k++) { out[cnt].n[k] = n[k]; out[cnt].pos[k] = v[k] - 0.5 * dist * n[k]; }
    cnt++;
  }
  return cnt;
}

/* dispatch one candidate pair (geom types ordered type1 <= type2) */
static int collide_geoms(const mgx_model_desc *m, ref_data *d, int g1, int g2, double margin, rcon *out) {
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const double *p1 = d->geom_xpos + 3 * g1, *m1 = d->geom_xmat + 9 * g1, *s1 = m->geom_size + 3 * g1;
  const double *p2 = d->geom_xpos + 3 * g2, *m2 = d->geom_xmat + 9 * g2, *s2 = m->geom_size + 3 * g2;
  /* bounding-sphere cull (mid-phase; no effect on results) */
  if (t1 != GPLANE) {
    double dv[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    if (norm3(dv) > m->geom_rbound[g1] + m->geom_rbound[g2] + margin) return 0;
  }
  if (t1 == GSPHERE && t2 == GSPHERE) return sph_sph_raw(p1, m1, s1[0], p2, m2, s2[0], margin, out);
  if (t1 == GSPHERE && t2 == GCAPSULE) return sphere_capsule(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GCAPSULE && t2 == GCAPSULE) return capsule_capsule(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GSPHERE && t2 == GBOX) return sphere_box_core(p1, s1[0], p2, m2, s2, margin, out);
  if (t1 == GCAPSULE && t2 == GBOX) return capsule_box(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GBOX && t2 == GBOX) {
    int n = box_box(p1, m1, s1, p2, m2, s2, margin, out);
    g_np_stats[5 + n]++;
    return n;
  }
  if (t1 == GPLANE && t2 == GSPHERE) return plane_sphere(p1, m1, p2, s2[0], margin, out);
  if (t1 == GPLANE && t2 == GCAPSULE) {
    double a[3], b[3];
    seg_ends(p2, m2, s2[1], a, b);
    int n = plane_sphere(p1, m1, a, s2[0], margin, out);
    n += plane_sphere(p1, m1, b, s2[0], margin, out + n);
    return n;
  }
  if (t1 == GPLANE && t2 == GBOX) return plane_box(p1, m1, p2, m2, s2, margin, out);
  if (t1 == GSPHERE && t2 == GCYLINDER) return sphere_cyl_core(p1, s1[0], p2, m2, s2, margin, out);
  if (t1 == GCAPSULE && t2 == GCYLINDER) return capsule_cyl(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GCYLINDER && t2 == GBOX) return cyl_box(p1, m1, s1, p2, m2, s2, margin, out);
  if (t1 == GCYLINDER && t2 == GCYLINDER) return cyl_cyl(p1, m1, s1, p2, m2, s2, margin, out);
  return 0; /* unsupported pair types (plane-cylinder, ellipsoid): no task has them */
}

static int add_contacts(const mgx_model_desc *m, ref_data *d, int pi, rcon *rc, int n) {
  int g1 = m->pair_geom[2 * pi], g2 = m->pair_geom[2 * pi + 1];
  for (int c = 0; c < n; c++) {
    int k = d->ncon[0];
    if (k >= d->ncon_max) return 0;
    d->con_dist[k] = rc[c].dist;
    memcpy(d->con_pos + 3 * k, rc[c].pos, 3 * sizeof(double));
    double *f = d->con_frame + 9 * k;
    f[0] = rc[c].n[0]; f[1] = rc[c].n[1]; f[2] = rc[c].n[2];
    make_frame(f);
    memcpy(d->con_friction + 5 * k, m->pair_friction + 5 * pi, 5 * sizeof(double));
    d->con_includemargin[k] = m->pair_margin[pi] - m->pair_gap[pi];
    memcpy(d->con_solref + 2 * k, m->pair_solref + 2 * pi, 2 * sizeof(double));
    memcpy(d->con_solimp + 5 * k, m->pair_solimp + 5 * pi, 5 * sizeof(double));
    d->con_geom[2 * k] = g1; d->con_geom[2 * k + 1] = g2;
    d->con_dim[k] = m->pair_condim[pi];
    d->con_pair[k] = pi;
    d->ncon[0]++;
  }
  return n;
}

int ref_collide_pair(const mgx_model_desc *m, ref_data *d, int pi) {
  rcon rc[MAXCONPAIR];
  int n = collide_geoms(m, d, m->pair_geom[2 * pi], m->pair_geom[2 * pi + 1], m->pair_margin[pi], rc);
  return add_contacts(m, d, pi, rc, n);
}

/* mj_collision [ext]: candidate pairs already in MuJoCo order (explicit, then sorted body pairs) */
static void collision(const mgx_model_desc *m, ref_data *d) {
  d->ncon[0] = 0;
  for (int pi = 0; pi < m->npair; pi++) ref_collide_pair(m, d, pi);
}

/* ====================================================================== constraints */
static void getimpedance(const double *solimp, double pos, double margin, double *imp) {
  double d0 = clampd(solimp[0], MINIMP, MAXIMP), d1 = clampd(solimp[1], MINIMP, MAXIMP);
  double width = solimp[2], mid = solimp[3], power = solimp[4];
  if (d0 == d1 || width <= MINVAL) { *imp = 0.5 * (d0 + d1); return; }
  double x = (pos - margin) / width;
  if (x < 0) x = -x;
  if (x >= 1 || x <= 0) { *imp = x >= 1 ? d1 : d0; return; }
  double y;
  if (power == 1) y = x;
  else if (x <= mid) y = pow(x, power) / pow(mid, power - 1);
  else y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  *imp = d0 + y * (d1 - d0);
}

static int add_row(ref_data *d, int type, int id, double pos, double margin, double diag) {
  int r = d->nefc[0];
  if (r >= d->nefc_max) return -1;
  d->efc_type[r] = type; d->efc_id[r] = id; d->efc_pos[r] = pos; d->efc_margin[r] = margin;
  d->efc_diagApprox[r] = diag;
  memset(d->efc_J + (size_t)r * d->nv, 0, sizeof(double) * d->nv);
  d->nefc[0]++;
  return r;
}

/* mj_makeConstraint: joint limits (mj_instantiateLimit) then contacts
 * (mj_instantiateContact, pyramidal cone) [ext] */
static void make_constraint(const mgx_model_desc *m, ref_data *d) {
  int nv = m->nv;
  d->nefc[0] = 0;
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j]) continue;
    int t = m->jnt_type[j];
    if (t != JHINGE && t != JSLIDE) continue;
    double val = d->qpos[m->jnt_qposadr[j]], margin = m->jnt_margin[j];
    for (int side = -1; side <= 1; side += 2) {
      double dist = side * (m->jnt_range[2 * j + (side + 1) / 2] - val);
      if (dist < margin) {
        int r = add_row(d, C_LIMIT_JOINT, j, dist, margin, m->dof_invweight0[m->jnt_dofadr[j]]);
        if (r < 0) return;
        d->efc_J[(size_t)r * nv + m->jnt_dofadr[j]] = -side;
      }
    }
  }
  double *jp1 = d->scratch, *jp2 = jp1 + 3 * nv, *jd = jp2 + 3 * nv;
  for (int c = 0; c < d->ncon[0]; c++) {
    int g1 = d->con_geom[2 * c], g2 = d->con_geom[2 * c + 1];
    int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
    int dim = d->con_dim[c];
    const double *fr = d->con_frame + 9 * c, *mu = d->con_friction + 5 * c;
    jac(m, d, jp1, NULL, d->con_pos + 3 * c, b1);
    jac(m, d, jp2, NULL, d->con_pos + 3 * c, b2);
    for (int k = 0; k < 3 * nv; k++) jd[k] = jp2[k] - jp1[k];
    double tran = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
    double rot = m->body_invweight0[2 * b1 + 1] + m->body_invweight0[2 * b2 + 1];
    /* contact-frame rows: cj[0] normal, cj[1..2] tangents (translational); cj[3] torsional,
       cj[4..5] rolling (rotational Jacobian on the normal / tangents) for condim 4 and 6 */
    double *cj = jd + 3 * nv;
    for (int a = 0; a < 3; a++)
      for (int k = 0; k < nv; k++)
        cj[a * nv + k] = fr[3 * a] * jd[k] + fr[3 * a + 1] * jd[nv + k] + fr[3 * a + 2] * jd[2 * nv + k];
    if (dim > 3) {
      double *jr1 = cj + 6 * nv, *jr2 = jr1 + 3 * nv;
      jac(m, d, jp1, jr1, d->con_pos + 3 * c, b1);
      jac(m, d, jp2, jr2, d->con_pos + 3 * c, b2);
      for (int k = 0; k < 3 * nv; k++) jr2[k] -= jr1[k];
      for (int a = 0; a < 3; a++)
        for (int k = 0; k < nv; k++)
          cj[(3 + a) * nv + k] = fr[3 * a] * jr2[k] + fr[3 * a + 1] * jr2[nv + k] + fr[3 * a + 2] * jr2[2 * nv + k];
    }
    if (dim == 1) {
      int r = add_row(d, C_CONTACT_FRICTIONLESS, c, d->con_dist[c], d->con_includemargin[c], tran);
      if (r < 0) return;
      memcpy(d->efc_J + (size_t)r * nv, cj, sizeof(double) * nv);
    } else {
      /* pyramid edges J_n +- mu_k J_k, k = 1 .. dim-1, in MuJoCo's order; diagApprox uses the
         translational weight for the two sliding directions and the rotational one for spin
         and rolling [ext] */
      for (int k = 1; k < dim; k++)
        for (int sgn = 0; sgn < 2; sgn++) {
          double f = mu[k - 1];
          int r = add_row(d, C_CONTACT_PYRAMIDAL, c, d->con_dist[c], d->con_includemargin[c],
                          tran + f * f * (k < 3 ? tran : rot));
          if (r < 0) return;
          double s = sgn ? -f : f;
          for (int q = 0; q < nv; q++) d->efc_J[(size_t)r * nv + q] = cj[q] + s * cj[k * nv + q];
        }
    }
  }
}

/* mj_makeImpedance: K, B, imp, R, D per row [ext] */
static void make_impedance(const mgx_model_desc *m, ref_data *d) {
  for (int r = 0; r < d->nefc[0]; r++) {
    const double *solref, *solimp;
    if (d->efc_type[r] == C_LIMIT_JOINT) {
      solref = m->jnt_solref + 2 * d->efc_id[r];
      solimp = m->jnt_solimp + 5 * d->efc_id[r];
    } else {
      solref = d->con_solref + 2 * d->efc_id[r];
      solimp = d->con_solimp + 5 * d->efc_id[r];
    }
    double imp;
    getimpedance(solimp, d->efc_pos[r], d->efc_margin[r], &imp);
    double dmax = clampd(solimp[1], MINIMP, MAXIMP), K, B;
    if (solref[0] > 0) {
      double tc = solref[0], dr = solref[1];
      if (tc < 2 * m->timestep) tc = 2 * m->timestep; /* refsafe */
      K = 1 / (dmax * dmax * tc * tc * dr * dr);
      B = 2 / (dmax * tc);
    } else {
      K = -solref[0] / (dmax * dmax);
      B = -solref[1] / dmax;
    }
    d->efc_KBIP[4 * r] = K; d->efc_KBIP[4 * r + 1] = B; d->efc_KBIP[4 * r + 2] = imp; d->efc_KBIP[4 * r + 3] = 0;
    double R = (1 - imp) * d->efc_diagApprox[r] / imp;
    d->efc_R[r] = R > MINVAL ? R : MINVAL;
    d->efc_D[r] = 1 / d->efc_R[r];
  }
}

/* mj_projectConstraint: AR = J M^-1 J' + diag(R) (dense) [ext] */
static void project_constraint(const mgx_model_desc *m, ref_data *d) {
  int nv = m->nv, ne = d->nefc[0];
  double *MinvJT = d->scratch; /* [ne][nv] */
  for (int r = 0; r < ne; r++) {
    memcpy(MinvJT + (size_t)r * nv, d->efc_J + (size_t)r * nv, sizeof(double) * nv);
    solve_ld(m, d->qLD, d->qLDiagInv, MinvJT + (size_t)r * nv);
  }
  for (int r = 0; r < ne; r++)
    for (int c = 0; c < ne; c++) {
      double s = 0;
      for (int k = 0; k < nv; k++) s += d->efc_J[(size_t)r * nv + k] * MinvJT[(size_t)c * nv + k];
      d->efc_AR[(size_t)r * ne + c] = s + (r == c ? d->efc_R[r] : 0);
    }
}

/* ====================================================================== velocity stage */
static void crossmotion(double *res, const double *v, const double *u) {
  res[0] = -v[2] * u[1] + v[1] * u[2];
  res[1] = v[2] * u[0] - v[0] * u[2];
  res[2] = -v[1] * u[0] + v[0] * u[1];
  res[3] = -v[2] * u[4] + v[1] * u[5];
  res[4] = v[2] * u[3] - v[0] * u[5];
  res[5] = -v[1] * u[3] + v[0] * u[4];
  res[3] += -v[5] * u[1] + v[4] * u[2];
  res[4] += v[5] * u[0] - v[3] * u[2];
  res[5] += -v[4] * u[0] + v[3] * u[1];
}
static void crossforce(double *res, const double *v, const double *f) {
  res[0] = -v[2] * f[1] + v[1] * f[2];
  res[1] = v[2] * f[0] - v[0] * f[2];
  res[2] = -v[1] * f[0] + v[0] * f[1];
  res[3] = -v[2] * f[4] + v[1] * f[5];
  res[4] = v[2] * f[3] - v[0] * f[5];
  res[5] = -v[1] * f[3] + v[0] * f[4];
  res[0] += -v[5] * f[4] + v[4] * f[5];
  res[1] += v[5] * f[3] - v[3] * f[5];
  res[2] += -v[4] * f[3] + v[3] * f[4];
}

/* mj_comVel [ext] */
static void comvel(const mgx_model_desc *m, ref_data *d) {
  memset(d->cvel, 0, 6 * sizeof(double));
  for (int i = 1; i < m->nbody; i++) {
    double cvel[6];
    memcpy(cvel, d->cvel + 6 * m->body_parentid[i], sizeof cvel);
    int bda = m->body_dofadr[i], nd = m->body_dofnum[i];
    for (int j = 0; j < nd; j++) {
      int dof = bda + j, t = m->jnt_type[m->dof_jntid[dof]];
      if (t == JFREE) {
        for (int k = 0; k < 18; k++) d->cdof_dot[6 * dof + k] = 0;
        for (int q = 0; q < 3; q++)
          for (int k = 0; k < 6; k++) cvel[k] += d->cdof[6 * (dof + q) + k] * d->qvel[dof + q];
        for (int q = 3; q < 6; q++) crossmotion(d->cdof_dot + 6 * (dof + q), cvel, d->cdof + 6 * (dof + q));
        for (int q = 3; q < 6; q++)
          for (int k = 0; k < 6; k++) cvel[k] += d->cdof[6 * (dof + q) + k] * d->qvel[dof + q];
        j += 5;
      } else if (t == JBALL) {
        for (int q = 0; q < 3; q++) crossmotion(d->cdof_dot + 6 * (dof + q), cvel, d->cdof + 6 * (dof + q));
        for (int q = 0; q < 3; q++)
          for (int k = 0; k < 6; k++) cvel[k] += d->cdof[6 * (dof + q) + k] * d->qvel[dof + q];
        j += 2;
      } else {
        crossmotion(d->cdof_dot + 6 * dof, cvel, d->cdof + 6 * dof);
        for (int k = 0; k < 6; k++) cvel[k] += d->cdof[6 * dof + k] * d->qvel[dof];
      }
    }
    memcpy(d->cvel + 6 * i, cvel, sizeof cvel);
  }
}

/* mj_passive: joint springs (hinge/slide) and dof damping [ext] */
static void passive(const mgx_model_desc *m, ref_data *d) {
  for (int k = 0; k < m->nv; k++) d->qfrc_passive[k] = -m->dof_damping[k] * d->qvel[k];
  for (int j = 0; j < m->njnt; j++) {
    double st = m->jnt_stiffness[j];
    if (st == 0) continue;
    int t = m->jnt_type[j], a = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (t == JHINGE || t == JSLIDE) d->qfrc_passive[da] -= st * (d->qpos[a] - m->qpos_spring[a]);
    else if (t == JFREE) for (int k = 0; k < 3; k++) d->qfrc_passive[da + k] -= st * (d->qpos[a + k] - m->qpos_spring[a + k]);
  }
}

/* mj_rne with flg_acc = 0: qfrc_bias = C(q, v) + gravity [ext] */
static void rne(const mgx_model_desc *m, ref_data *d) {
  int nb = m->nbody;
  double *cacc = d->scratch, *cfrc = cacc + 6 * nb, tmp[6], tmp1[6];
  memset(cacc, 0, 6 * sizeof(double));
  for (int k = 0; k < 3; k++) cacc[3 + k] = -m->gravity[k];
  for (int i = 1; i < nb; i++) {
    int bda = m->body_dofadr[i], nd = m->body_dofnum[i], p = m->body_parentid[i];
    for (int k = 0; k < 6; k++) cacc[6 * i + k] = cacc[6 * p + k];
    for (int j = 0; j < nd; j++)
      for (int k = 0; k < 6; k++) cacc[6 * i + k] += d->cdof_dot[6 * (bda + j) + k] * d->qvel[bda + j];
    mulinertvec(cfrc + 6 * i, d->cinert + 10 * i, cacc + 6 * i);
    mulinertvec(tmp, d->cinert + 10 * i, d->cvel + 6 * i);
    crossforce(tmp1, d->cvel + 6 * i, tmp);
    for (int k = 0; k < 6; k++) cfrc[6 * i + k] += tmp1[k];
  }
  memset(cfrc, 0, 6 * sizeof(double));
  for (int i = nb - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p) for (int k = 0; k < 6; k++) cfrc[6 * p + k] += cfrc[6 * i + k];
  }
  for (int k = 0; k < m->nv; k++) d->qfrc_bias[k] = dot6(d->cdof + 6 * k, cfrc + 6 * m->dof_bodyid[k]);
}

/* mj_fwdActuation for joint transmissions [ext] */
static void actuation(const mgx_model_desc *m, ref_data *d) {
  memset(d->qfrc_actuator, 0, sizeof(double) * m->nv);
  for (int u = 0; u < m->nu; u++) {
    int j = m->actuator_trnid[u];
    double ctrl = d->ctrl[u];
    if (m->actuator_ctrllimited[u]) ctrl = clampd(ctrl, m->actuator_ctrlrange[2 * u], m->actuator_ctrlrange[2 * u + 1]);
    double g = m->actuator_gear[u];
    double len = g * d->qpos[m->jnt_qposadr[j]], vel = g * d->qvel[m->jnt_dofadr[j]];
    const double *gp = m->actuator_gainprm + 3 * u, *bp = m->actuator_biasprm + 3 * u;
    double f = gp[0] * ctrl + bp[0] + bp[1] * len + bp[2] * vel;
    if (m->actuator_forcelimited[u]) f = clampd(f, m->actuator_forcerange[2 * u], m->actuator_forcerange[2 * u + 1]);
    d->actuator_force[u] = f;
    d->qfrc_actuator[m->jnt_dofadr[j]] += g * f;
  }
}

/* mj_xfrcAccumulate: qfrc += J(xipos)' * xfrc_applied [ext] */
static void xfrc_accumulate(const mgx_model_desc *m, ref_data *d, double *qfrc) {
  int nv = m->nv;
  double *jp = d->scratch + 12 * m->nbody, *jr = jp + 3 * nv;
  for (int i = 1; i < m->nbody; i++) {
    const double *f = d->xfrc_applied + 6 * i;
    if (!f[0] && !f[1] && !f[2] && !f[3] && !f[4] && !f[5]) continue;
    jac(m, d, jp, jr, d->xipos + 3 * i, i);
    for (int k = 0; k < nv; k++)
      qfrc[k] += jp[k] * f[0] + jp[nv + k] * f[1] + jp[2 * nv + k] * f[2] +
                 jr[k] * f[3] + jr[nv + k] * f[4] + jr[2 * nv + k] * f[5];
  }
}

/* ====================================================================== solver */
/* mj_constraintUpdate restricted to limit/contact rows (one-sided) */
static void constraint_force_from_jar(ref_data *d, const double *jar) {
  for (int r = 0; r < d->nefc[0]; r++) d->efc_force[r] = jar[r] < 0 ? -d->efc_D[r] * jar[r] : 0;
}

/* ---- mj_solNewton [ext]: the primal problem over accelerations a,
 *   minimise  0.5 (a - a0)' M (a - a0) + sum_r s_r(J_r a - aref_r),
 *   s_r(x) = 0.5 D_r x^2 for x < 0 (contacts, pyramid rows and limits are one-sided), D = 1/R,
 * whose minimiser is unique (M and D positive). Each iteration: H = M + J_A' D_A J_A over the
 * active rows, dense Cholesky, p = -H^-1 g, then the exact line search on the convex
 * piecewise-quadratic f(alpha) (safeguarded Newton on the monotone piecewise-linear f').
 * Warmstart from qacc_warmstart when its cost is below qacc_smooth's; stop on scaled
 * improvement or gradient below tolerance, or after `iterations`. The converged minimiser is
 * what any exact solver returns, so this restatement pins the device Newton solver. */
static double newton_cost(const mgx_model_desc *m, ref_data *d, const double *a, const double *M, double *x,
                          double *grad) {
  int nv = m->nv, ne = d->nefc[0];
  double c = 0;
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int k = 0; k < nv; k++) s += M[i * nv + k] * (a[k] - d->qacc_smooth[k]);
    if (grad) grad[i] = s;
    c += 0.5 * (a[i] - d->qacc_smooth[i]) * s;
  }
  for (int r = 0; r < ne; r++) {
    const double *J = d->efc_J + (size_t)r * nv;
    double s = -d->efc_aref[r];
    for (int k = 0; k < nv; k++) s += J[k] * a[k];
    x[r] = s;
    if (s < 0) {
      double Dr = 1 / d->efc_R[r];
      c += 0.5 * Dr * s * s;
      if (grad) for (int k = 0; k < nv; k++) grad[k] += Dr * s * J[k];
    }
  }
  return c;
}

/* Newton diagnostics (ref_newton_stats): solves, iterations, active rows summed over iterations,
   rows whose active state changed since the previous iteration of the same solve */
static long g_newton_stats[4];
void ref_newton_stats(long *out, int reset) {
  for (int k = 0; k < 4; k++) out[k] = g_newton_stats[k];
  if (reset)
    for (int k = 0; k < 4; k++) g_newton_stats[k] = 0;
}

static void newton_solve(const mgx_model_desc *m, ref_data *d) {
  int nv = m->nv, ne = d->nefc[0];
  unsigned char *prev_act = calloc(ne > 0 ? ne : 1, 1);
  g_newton_stats[0]++;
  double *M = malloc(sizeof(double) * (3 * nv * nv + 6 * nv + 3 * ne));
  double *H = M + nv * nv, *a = H + nv * nv, *g = a + nv, *p = g + nv, *Mp = p + nv, *tmp = Mp + nv;
  double *x = tmp + 2 * nv, *jp = x + ne, *xt = jp + ne;
  (void)xt;
  /* dense M from the tree-sparse qM */
  memset(M, 0, sizeof(double) * nv * nv);
  for (int i = 0; i < nv; i++) {
    int adr = m->dof_Madr[i], t = 0;
    for (int j = i; j >= 0; j = m->dof_parentid[j], t++) {
      M[i * nv + j] = d->qM[adr + t];
      M[j * nv + i] = d->qM[adr + t];
    }
  }
  double scale = 1 / (m->meaninertia * (nv > 1 ? nv : 1));
  /* warmstart */
  double c0 = newton_cost(m, d, d->qacc_smooth, M, x, NULL);
  double cw = newton_cost(m, d, d->qacc_warmstart, M, x, NULL);
  memcpy(a, cw < c0 ? d->qacc_warmstart : d->qacc_smooth, sizeof(double) * nv);
  newton_cost(m, d, a, M, x, g);
  int iter = 0;
  /* mj_solNewton's loop order [ext]: every iteration updates, then tests the scaled improvement
     and the scaled gradient at the new point, so at least one iteration always runs */
  while (iter < m->iterations) {
    g_newton_stats[1]++;
    for (int r = 0; r < ne; r++) {
      const unsigned char act = x[r] < 0;
      g_newton_stats[2] += act;
      if (iter > 0 && act != prev_act[r]) g_newton_stats[3]++;
      prev_act[r] = act;
    }
    /* H = M + J_A' D_A J_A, Cholesky (lower, in place) */
    memcpy(H, M, sizeof(double) * nv * nv);
    for (int r = 0; r < ne; r++) {
      if (x[r] >= 0) continue;
      const double *J = d->efc_J + (size_t)r * nv;
      double Dr = 1 / d->efc_R[r];
      for (int i = 0; i < nv; i++) {
        if (J[i] == 0) continue;
        for (int k = 0; k <= i; k++) H[i * nv + k] += Dr * J[i] * J[k];
      }
    }
    for (int k = 0; k < nv; k++) {
      double s = H[k * nv + k];
      for (int j = 0; j < k; j++) s -= H[k * nv + j] * H[k * nv + j];
      s = sqrt(s > MINVAL ? s : MINVAL);
      H[k * nv + k] = s;
      const double inv = 1 / s; /* mju_cholFactor scales the column by 1 / L_kk */
      for (int i = k + 1; i < nv; i++) {
        double t = H[i * nv + k];
        for (int j = 0; j < k; j++) t -= H[i * nv + j] * H[k * nv + j];
        H[i * nv + k] = t * inv;
      }
    }
    for (int i = 0; i < nv; i++) { /* L y = -g */
      double s = -g[i];
      for (int j = 0; j < i; j++) s -= H[i * nv + j] * tmp[j];
      tmp[i] = s / H[i * nv + i];
    }
    for (int i = nv - 1; i >= 0; i--) { /* L' p = y */
      double s = tmp[i];
      for (int j = i + 1; j < nv; j++) s -= H[j * nv + i] * p[j];
      p[i] = s / H[i * nv + i];
    }
    /* exact line search: f'(al) = (a-a0)'Mp + al p'Mp + sum_{x+al jp<0} D (x + al jp) jp */
    double g0 = 0, pMp = 0;
    for (int i = 0; i < nv; i++) {
      double s = 0;
      for (int k = 0; k < nv; k++) s += M[i * nv + k] * p[k];
      Mp[i] = s;
      g0 += (a[i] - d->qacc_smooth[i]) * s;
      pMp += p[i] * s;
    }
    for (int r = 0; r < ne; r++) {
      const double *J = d->efc_J + (size_t)r * nv;
      double s = 0;
      for (int k = 0; k < nv; k++) s += J[k] * p[k];
      jp[r] = s;
    }
    /* line search, MuJoCo's stop rule [ext]: the cost along p is convex piecewise quadratic; the
       first point is the Newton step from alpha = 0, then safeguarded Newton steps inside the
       bracket [lo, hi] (bisection when a step leaves it) until |f'(alpha)| < gtol =
       tolerance * ls_tolerance * |p| * meaninertia * max(1, nv), at most ls_iterations = 50
       evaluations (MuJoCo defaults ls_tolerance 0.01, ls_iterations 50; no model sets them) */
    double snorm = 0;
    for (int k = 0; k < nv; k++) snorm += p[k] * p[k];
    snorm = sqrt(snorm);
    double al = 0;
    if (snorm >= MINVAL) {
      const double gtol = m->tolerance * LS_TOLERANCE * snorm * m->meaninertia * (nv > 1 ? nv : 1);
      double d1 = g0, d2 = pMp;
      for (int r = 0; r < ne; r++)
        if (x[r] < 0) {
          double Dr = 1 / d->efc_R[r];
          d1 += Dr * x[r] * jp[r];
          d2 += Dr * jp[r] * jp[r];
        }
      al = -d1 / d2;
      double lo = 0, hi = 1e300;
      for (int ls = 0; ls < LS_ITERATIONS; ls++) {
        d1 = g0 + al * pMp;
        d2 = pMp;
        for (int r = 0; r < ne; r++) {
          double xr = x[r] + al * jp[r];
          if (xr < 0) {
            double Dr = 1 / d->efc_R[r];
            d1 += Dr * xr * jp[r];
            d2 += Dr * jp[r] * jp[r];
          }
        }
        if (fabs(d1) < gtol) break;
        if (d1 < 0) lo = al; else hi = al;
        double nxt = d2 > 0 ? al - d1 / d2 : 2 * al;
        if (!(nxt > lo && nxt < hi)) nxt = hi < 1e300 ? 0.5 * (lo + hi) : 2 * al;
        const int stall = fabs(nxt - al) <= 1e-15 * (1 + fabs(al));  /* no change in floating point */
        al = nxt;
        if (stall) break;
      }
    }
    /* the improvement cost(old) - cost(new) evaluated term by term along the step (the Gauss
       term al g0 + al^2 pMp / 2 and each row's change of s_r): algebraically MuJoCo's
       difference of totals, which at ~1e10 costs (construction states) rounds to 0 or a few
       ulps and would let rounding decide the stop test; the device evaluates the same terms */
    double dec = al * g0 + 0.5 * al * al * pMp;
    for (int r = 0; r < ne; r++) {
      const double xo = x[r], xn = x[r] + al * jp[r], Dr = 1 / d->efc_R[r];
      if (xo < 0 && xn < 0) dec += 0.5 * Dr * (al * jp[r]) * (xo + xn);
      else if (xo < 0) dec -= 0.5 * Dr * xo * xo;
      else if (xn < 0) dec += 0.5 * Dr * xn * xn;
    }
    for (int k = 0; k < nv; k++) a[k] += al * p[k];
    newton_cost(m, d, a, M, x, g);
    double improvement = -scale * dec;
    iter++;
    double gn = 0;
    for (int k = 0; k < nv; k++) gn += g[k] * g[k];
    if (improvement < m->tolerance || scale * sqrt(gn) < m->tolerance) break;
  }
  d->solver_niter[0] = iter;
  free(prev_act);
  memcpy(d->qacc, a, sizeof(double) * nv);
  for (int r = 0; r < ne; r++) d->efc_force[r] = x[r] < 0 ? -x[r] / d->efc_R[r] : 0;
  memset(d->qfrc_constraint, 0, sizeof(double) * nv);
  for (int r = 0; r < ne; r++)
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] += d->efc_J[(size_t)r * nv + k] * d->efc_force[r];
  free(M);
}

/* mj_fwdConstraint with warmstart + mj_solPGS (or mj_solNewton) [ext] */
static void fwd_constraint(const mgx_model_desc *m, ref_data *d) {
  int nv = m->nv, ne = d->nefc[0];
  if (!ne) {
    memcpy(d->qacc, d->qacc_smooth, sizeof(double) * nv);
    memset(d->qfrc_constraint, 0, sizeof(double) * nv);
    d->solver_niter[0] = 0;
    return;
  }
  if (m->solver == 2) {
    newton_solve(m, d);
    return;
  }
  double *jar = d->scratch, *ARf = jar + ne;
  /* efc_b = J qacc_smooth - aref */
  for (int r = 0; r < ne; r++) {
    double s = 0;
    for (int k = 0; k < nv; k++) s += d->efc_J[(size_t)r * nv + k] * d->qacc_smooth[k];
    d->efc_b[r] = s - d->efc_aref[r];
  }
  /* warmstart: forces implied by qacc_warmstart; zero if its dual cost is positive */
  for (int r = 0; r < ne; r++) {
    double s = 0;
    for (int k = 0; k < nv; k++) s += d->efc_J[(size_t)r * nv + k] * d->qacc_warmstart[k];
    jar[r] = s - d->efc_aref[r];
  }
  constraint_force_from_jar(d, jar);
  double cost = 0;
  for (int r = 0; r < ne; r++) {
    double s = 0;
    for (int c = 0; c < ne; c++) s += d->efc_AR[(size_t)r * ne + c] * d->efc_force[c];
    ARf[r] = s;
    cost += d->efc_force[r] * (d->efc_b[r] + 0.5 * s);
  }
  if (cost > 0) memset(d->efc_force, 0, sizeof(double) * ne);
  /* PGS sweeps */
  double scale = 1 / (m->meaninertia * (nv > 1 ? nv : 1));
  int iter = 0;
  while (iter < m->iterations) {
    double improvement = 0;
    for (int r = 0; r < ne; r++) {
      const double *Ar = d->efc_AR + (size_t)r * ne;
      double res = d->efc_b[r];
      if (d->pgs_reverse)
        for (int c = ne - 1; c >= 0; c--) res += Ar[c] * d->efc_force[c];
      else
        for (int c = 0; c < ne; c++) res += Ar[c] * d->efc_force[c];
      double Arr = Ar[r], old = d->efc_force[r];
      double f = old - res / Arr;
      if (d->efc_type[r] >= C_LIMIT_JOINT && f < 0) f = 0;
      double delta = f - old;
      double change = 0.5 * delta * delta * Arr + delta * res;
      if (change > 1e-10) { f = old; change = 0; }
      d->efc_force[r] = f;
      improvement -= change;
    }
    iter++;
    if (improvement * scale < m->tolerance) break;
  }
  d->solver_niter[0] = iter;
  /* qfrc_constraint = J' f ; qacc = qacc_smooth + M^-1 qfrc_constraint */
  memset(d->qfrc_constraint, 0, sizeof(double) * nv);
  for (int r = 0; r < ne; r++)
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] += d->efc_J[(size_t)r * nv + k] * d->efc_force[r];
  double *tmp = d->scratch;
  memcpy(tmp, d->qfrc_constraint, sizeof(double) * nv);
  solve_ld(m, d->qLD, d->qLDiagInv, tmp);
  for (int k = 0; k < nv; k++) d->qacc[k] = d->qacc_smooth[k] + tmp[k];
}

/* ====================================================================== forward / step */
void ref_forward(const mgx_model_desc *m, ref_data *d) {
  int nv = m->nv;
  /* mj_fwdPosition */
  kinematics(m, d);
  compos(m, d);
  crb(m, d);
  factor_ld(m, d->qM, d->qLD, d->qLDiagInv);
  collision(m, d);
  make_constraint(m, d);
  make_impedance(m, d);
  project_constraint(m, d);
  /* mj_fwdVelocity */
  comvel(m, d);
  passive(m, d);
  for (int r = 0; r < d->nefc[0]; r++) { /* mj_referenceConstraint */
    double s = 0;
    for (int k = 0; k < nv; k++) s += d->efc_J[(size_t)r * nv + k] * d->qvel[k];
    d->efc_vel[r] = s;
    d->efc_aref[r] = -d->efc_KBIP[4 * r + 1] * s -
                     d->efc_KBIP[4 * r] * d->efc_KBIP[4 * r + 2] * (d->efc_pos[r] - d->efc_margin[r]);
  }
  rne(m, d);
  /* mj_fwdActuation, mj_fwdAcceleration */
  actuation(m, d);
  for (int k = 0; k < nv; k++)
    d->qfrc_smooth[k] = d->qfrc_passive[k] - d->qfrc_bias[k] + d->qfrc_applied[k] + d->qfrc_actuator[k];
  xfrc_accumulate(m, d, d->qfrc_smooth);
  memcpy(d->qacc_smooth, d->qfrc_smooth, sizeof(double) * nv);
  solve_ld(m, d->qLD, d->qLDiagInv, d->qacc_smooth);
  /* mj_fwdConstraint */
  fwd_constraint(m, d);
}

/* mju_quatIntegrate */
static void quat_integrate(double *q, const double *w, double h) {
  double ax[3] = {w[0], w[1], w[2]}, qr[4];
  double ang = h * normalize3(ax);
  axisangle2quat(qr, ax, ang);
  normalize4(q);
  mulquat(q, q, qr);
}

/* mj_integratePos [ext] */
static void integrate_pos(const mgx_model_desc *m, double *qpos, const double *qvel, double h) {
  for (int j = 0; j < m->njnt; j++) {
    int a = m->jnt_qposadr[j], da = m->jnt_dofadr[j], t = m->jnt_type[j];
    if (t == JFREE) {
      for (int k = 0; k < 3; k++) qpos[a + k] += h * qvel[da + k];
      quat_integrate(qpos + a + 3, qvel + da + 3, h);
    } else if (t == JBALL) {
      quat_integrate(qpos + a, qvel + da, h);
    } else {
      qpos[a] += h * qvel[da];
    }
  }
}

/* mj_Euler with implicit joint damping:
 * qacc <- (M + h diag(damping))^-1 (qfrc_smooth + qfrc_constraint) [ext] */
static void euler(const mgx_model_desc *m, ref_data *d) {
  int nv = m->nv;
  double *qacc = d->scratch, *MH = qacc + nv, *MHinv = MH + m->nM;
  int damp = 0;
  for (int k = 0; k < nv; k++) if (m->dof_damping[k] > 0) damp = 1;
  if (!damp) memcpy(qacc, d->qacc, sizeof(double) * nv);
  else {
    memcpy(MH, d->qM, sizeof(double) * m->nM);
    for (int k = 0; k < nv; k++) MH[m->dof_Madr[k]] += m->timestep * m->dof_damping[k];
    factor_ld(m, MH, MH, MHinv);
    for (int k = 0; k < nv; k++) qacc[k] = d->qfrc_smooth[k] + d->qfrc_constraint[k];
    solve_ld(m, MH, MHinv, qacc);
  }
  for (int k = 0; k < nv; k++) d->qvel[k] += m->timestep * qacc[k];
  integrate_pos(m, d->qpos, d->qvel, m->timestep);
  d->time[0] += m->timestep;
}

/* mj_RungeKutta(m, d, 4) [ext]: classic RK4 Butcher tableau A = [.5; 0 .5; 0 0 1],
 * B = [1/6 1/3 1/3 1/6]. Stage i evaluates mj_forwardSkip at X[i] = X[0] '+' h sum_j A_ij X'[j]
 * (positions through integratePos); the final update is mj_advance with dX = sum_j B_j X'[j]:
 * qvel += h dX_acc, qpos = integratePos(qpos0, dX_vel, h). The forward-pass outputs left in
 * d (xpos, contacts, qacc) are those of the LAST stage evaluation, as in MuJoCo; the warmstart
 * saved for the next step is that last stage's qacc (mj_advance copies d->qacc). */
static void rk4(const mgx_model_desc *m, ref_data *d) {
  static const double A[9] = {0.5, 0, 0, 0, 0.5, 0, 0, 0, 1.0};
  static const double B[4] = {1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0};
  int nq = m->nq, nv = m->nv;
  double h = m->timestep, t0 = d->time[0];
  double *X[4], *F[4];
  double *buf = malloc(sizeof(double) * (4 * (nq + nv) + 4 * nv + 2 * nv));
  for (int i = 0; i < 4; i++) { X[i] = buf + i * (nq + nv); F[i] = buf + 4 * (nq + nv) + i * nv; }
  double *dX = buf + 4 * (nq + nv) + 4 * nv;
  memcpy(X[0], d->qpos, sizeof(double) * nq);
  memcpy(X[0] + nq, d->qvel, sizeof(double) * nv);
  memcpy(F[0], d->qacc, sizeof(double) * nv);
  for (int i = 1; i < 4; i++) {
    double C = 0;
    for (int j = 0; j < i; j++) C += A[(i - 1) * 3 + j];
    memset(dX, 0, sizeof(double) * 2 * nv);
    for (int j = 0; j < i; j++) {
      double a = A[(i - 1) * 3 + j];
      for (int k = 0; k < nv; k++) { dX[k] += a * X[j][nq + k]; dX[nv + k] += a * F[j][k]; }
    }
    memcpy(X[i], X[0], sizeof(double) * (nq + nv));
    integrate_pos(m, X[i], dX, h);
    for (int k = 0; k < nv; k++) X[i][nq + k] += h * dX[nv + k];
    memcpy(d->qpos, X[i], sizeof(double) * nq);
    memcpy(d->qvel, X[i] + nq, sizeof(double) * nv);
    d->time[0] = t0 + C * h;
    ref_forward(m, d);
    memcpy(F[i], d->qacc, sizeof(double) * nv);
  }
  memset(dX, 0, sizeof(double) * 2 * nv);
  for (int j = 0; j < 4; j++)
    for (int k = 0; k < nv; k++) { dX[k] += B[j] * X[j][nq + k]; dX[nv + k] += B[j] * F[j][k]; }
  d->time[0] = t0;
  memcpy(d->qpos, X[0], sizeof(double) * nq);
  memcpy(d->qvel, X[0] + nq, sizeof(double) * nv);
  /* mj_advance */
  memcpy(d->qacc_warmstart, d->qacc, sizeof(double) * nv);
  for (int k = 0; k < nv; k++) d->qvel[k] += h * dX[nv + k];
  integrate_pos(m, d->qpos, dX, h);
  d->time[0] += h;
  free(buf);
}

static int check_bad(const double *x, int n) {
  for (int i = 0; i < n; i++) if (isbad(x[i])) return 1;
  return 0;
}

/* mj_step: checkPos, checkVel, forward, checkAcc, then Euler or RK4 [ext] */
void ref_step(const mgx_model_desc *m, ref_data *d) {
  if (check_bad(d->qpos, m->nq)) { ref_reset(m, d); d->warning[0]++; }
  if (check_bad(d->qvel, m->nv)) { ref_reset(m, d); d->warning[0]++; }
  ref_forward(m, d);
  if (check_bad(d->qacc, m->nv)) {
    ref_reset(m, d);
    d->warning[0]++;
    ref_forward(m, d);
  }
  if (m->integrator == 1) {
    rk4(m, d);
    return;
  }
  memcpy(d->qacc_warmstart, d->qacc, sizeof(double) * m->nv);
  euler(m, d);
}
