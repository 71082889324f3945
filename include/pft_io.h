/*
 * pft_io.h -- snapshot / restart datasets of the intertrack (u, p, gl) state.
 *
 * The reference writes every snapshot with the NetCDF library in its classic format
 * (intertrack.c:2331 nc_create(..., NC_CLOBBER)) and reads one back for `icond_file` /
 * `continue_series` restarts (intertrack.c:1584-1669, 2040-2069).  NetCDF is not available in
 * this image, so libpft writes the same dataset with its own NetCDF-classic writer:
 *   - dimensions n3 = total_n3, n2, n1 (interior cells, grid_IO_mode 1, :2338-2340);
 *   - coordinate variables n3, n2, n1 (double): L3*(0.5+k)/total_n3, L2*(0.5+j)/n2, L1*(0.5+i)/n1
 *     (:2441-2443), then one double variable per model variable, u, p, gl, [n3][n2][n1] (:2354);
 *   - global attributes in the reference's order (:2382-2406): L1, L2, L3, the model parameters
 *     in param_info[] order (model.c:85-137), calc_mode (int), delta, tau, t, final_time,
 *     snapshot (int), total_snapshots (int), title (text).
 * Format: CDF-1 ("classic") when the file stays below 2 GiB, CDF-2 (64-bit offsets) above it
 * (the 800^3 case), readable by any NetCDF reader.  Data are big-endian, as the format requires.
 *
 * Multi-GPU: one shared file, no gather.  pft_snapshot_create() (one rank) writes the header,
 * the coordinates and sizes the file; after a barrier every rank writes its own Z-slab planes
 * with pft_snapshot_write_slab() at their offsets.  pft_snapshot_write() does both over the
 * current pft communicator.  Host layout of x is the reference's padded layout (pft_model.h).
 * Return codes: 0 OK; -1 I/O error (errno kept); -2 bad argument; -3 not a NetCDF classic file or
 * a variable/dimension missing; -4 dimensions differ from the grid.
 */
#ifndef PFT_IO_H
#define PFT_IO_H

#include "pft_model.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
	double t;               /* eqSystem.t */
	double tau;             /* eqSystem.h (the next step size) */
	double final_time;
	double delta;
	int snapshot, total_snapshots;
	int calc_mode;
	char title[256];        /* "Intertrack simulation (<comment>). Time: <t>" (:1129, :2405) */
	double L1, L2, L3;      /* read back from the dataset (written from the grid) */
} pft_snapshot_info;

/* header + coordinate variables, file sized to its final length; param = PFT_PARAM_COUNT values
   in pft_model.h order (written in param_info order); version 0 = automatic, 1 = CDF-1, 2 = CDF-2 */
int pft_snapshot_create(const char * path, const pft_grid * g, const double * param,
                        const pft_snapshot_info * info, int version);
/* this slab's interior planes of u, p, gl from the host padded array x */
int pft_snapshot_write_slab(const char * path, const pft_grid * g, const double * x);
/* create (rank 0) + barrier + write_slab (every rank) over the current communicator */
int pft_snapshot_write(const char * path, const pft_grid * g, const double * param,
                       const pft_snapshot_info * info, const double * x);

/* dimensions, attributes (info) and, if param != NULL, the model parameters of a dataset */
int pft_snapshot_read_info(const char * path, int * n1, int * n2, int * total_n3,
                           pft_snapshot_info * info, double * param);
/* this slab's interior planes into the host padded array x (ghost cells untouched) */
int pft_snapshot_read_slab(const char * path, const pft_grid * g, double * x);

/* the title the reference writes (:1129, :2405): "Intertrack simulation (%s). Time: %g" */
int pft_snapshot_title(char * buf, int size, const char * comment, double t);

#ifdef __cplusplus
}
#endif
#endif
