/*
 * pft_internal.h -- glue between libpft's model (intertrack_model.c) and solver (rk_solver.c).
 * Not part of the public ABI.
 */
#ifndef PFT_INTERNAL_H
#define PFT_INTERNAL_H

#include "../../include/pft_model.h"
#include "../../include/pft_hip.h"
#include "../../include/pft_comm.h"
#include "../../include/pft_solver.h"

/* 1 if f is one of the model's device right-hand sides for the configured calc_mode */
int pft_model_is_device_rhs(RK_RightHandSide f);
/* configured grid (0) or -3 if pft_model_configure() was not called on this thread */
int pft_model_get_grid(pft_grid * g);
/* device constants for the configured grid and parameters */
int pft_model_get_consts(pft_consts * c);
/* host u_noise field [k][j][i] of this slab, or NULL when u_noise_amp == 0 */
const double * pft_model_noise(void);

/* f1: the per-axis tables of the device initial condition (pft_slab_ic_default) for the
   configured slab, with or without the bead overlay; free(*store), free(*istore) afterwards */
int pft_model_ic_tables(pft_ic_tables * t, int with_beads, double ** store, int ** istore);

#endif
