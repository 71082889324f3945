/*
 * mock_intertrack.c -- TEST DRIVER for include/pft_equation_adapter.c (not part of libpft).
 *
 * Stands where apps/intertrack-hybrid-S-freezing/intertrack.c stands: it defines the driver
 * statics the model file reads (same names and types as intertrack.c:233-428), #includes the
 * adapter in place of equation.c (intertrack.c:633) and makes the driver's calls in the driver's
 * order -- MPI_Init, sizes (:1776-1800), `solution` (:1813), AllocPrecalcData (:1814), the
 * initial condition, PrecalculateData (:646), the chunk table (:2144-2157), the positional
 * eqSystem initialiser (:2163-2190), RK_MPI_SA_init (:2192), check_mem (:2208), solve (:2283),
 * RK_MPI_SA_cleanup (:2725), FreePrecalcData.  Then it writes the interior of u, p, gl.
 *
 *   mock_intertrack <params.txt> n1 n2 total_n3 L1 L2 L3 calc_mode tau tau_min delta final_time <out>
 * (under mpirun with several ranks each rank writes its own slab to <out>.<rank>)
 * params.txt: the 30 model parameters (model.c:44-59 order), one per line (C99 hex floats ok).
 * data/spheres_positions.txt must exist in the working directory (equation.c:35).
 */
#include <stdio.h>
#include <stdlib.h>
#include <mpi.h>
#include "RK_MPI_SAsolver.h"

/* ---- driver statics read by the model file ---- */
static int n1, n2, n3, total_n3, first_row;
static FLOAT L1, L2, L3;
static FLOAT model_parameters[30];
static FLOAT * param = model_parameters;
static FLOAT * solution;
static int calc_mode;
static int MPIrank, MPIprocs, MPImaster = 0;
static int * MPIrankmap;

#include "pft_equation_adapter.c"

int main(int argc, char ** argv)
{
	int i, j, k, q, c, N1, N2, N3, n_chunks, rc;
	long S;
	FLOAT tau, tau_min, delta, final_time, var_eps_mult[3] = {1.0, 1.0, 1.0};
	int * chunk_start, * chunk_size;
	FLOAT * chunk_eps_mult;
	FILE * f;

	MPI_Init(&argc, &argv);
	MPI_Comm_rank(MPI_COMM_WORLD, &MPIrank);
	MPI_Comm_size(MPI_COMM_WORLD, &MPIprocs);
	if(argc != 14) { fprintf(stderr, "usage: see header\n"); MPI_Abort(MPI_COMM_WORLD, 2); }
	MPIrankmap = (int *)malloc(MPIprocs * sizeof(int));
	for(i = 0; i < MPIprocs; i++) MPIrankmap[i] = i;
	f = fopen(argv[1], "r");
	for(i = 0; i < 30; i++) if(!f || fscanf(f, "%lf", model_parameters + i) != 1) MPI_Abort(MPI_COMM_WORLD, 3);
	fclose(f);
	n1 = atoi(argv[2]); n2 = atoi(argv[3]); total_n3 = atoi(argv[4]);
	L1 = strtod(argv[5], NULL); L2 = strtod(argv[6], NULL); L3 = strtod(argv[7], NULL);
	calc_mode = atoi(argv[8]);
	tau = strtod(argv[9], NULL); tau_min = strtod(argv[10], NULL);
	delta = strtod(argv[11], NULL); final_time = strtod(argv[12], NULL);

	pft_decompose(total_n3, MPIprocs, MPIrank, &n3, &first_row);
	N1 = n1 + 2 * bcond_thickness; N2 = n2 + 2 * bcond_thickness; N3 = n3 + 2 * bcond_thickness;
	S = (long)N1 * N2 * N3;
	solution = (FLOAT *)calloc(3 * S, sizeof(FLOAT));
	{
		/* the driver's CheckErrorAcrossRanks (intertrack.c:1814-1826): every rank learns of any
		   rank's allocation error and all of them exit */
		int err = !solution || AllocPrecalcData(), any = 0;
		MPI_Allreduce(&err, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
		if(any) {
			if(err) fprintf(stderr, "rank %d: AllocPrecalcData failed\n", MPIrank);
			MPI_Finalize();
			return 4;
		}
	}
	if(pft_model_ic_default(solution)) MPI_Abort(MPI_COMM_WORLD, 5);
	if(PrecalculateData(var_eps_mult)) { fprintf(stderr, "PrecalculateData failed\n"); MPI_Abort(MPI_COMM_WORLD, 6); }

	n_chunks = 3 * n2 * n3;
	chunk_start = (int *)malloc(n_chunks * sizeof(int));
	chunk_size = (int *)malloc(n_chunks * sizeof(int));
	chunk_eps_mult = (FLOAT *)malloc(n_chunks * sizeof(FLOAT));
	for(q = 0, c = 0; q < 3; q++)
		for(k = 0; k < n3; k++)
			for(j = 0; j < n2; j++, c++) {
				chunk_start[c] = (int)(q * S + (long)(k + bcond_thickness) * N1 * N2 + (j + bcond_thickness) * N1 + bcond_thickness);
				chunk_size[c] = n1;
				chunk_eps_mult[c] = var_eps_mult[q];
			}
	{
		RK_MEM_DIST mem_dist = { n_chunks, chunk_start, chunk_size, chunk_eps_mult };
		RK_MPI_S_SOLUTION eqSystem = {
			&mem_dist, 0.0, solution,
			MPIprocs == 1 ? mf_single : (MPIrank == 0 ? mf_bottom : (MPIrank == MPIprocs - 1 ? mf_top : mf_middle)),
			tau, tau_min, delta, DELTA_GLOBAL, NULL, NULL, 0, 0
		};
		if((rc = RK_MPI_SA_init(3 * (int)S, MPI_COMM_WORLD, MPImaster))) { fprintf(stderr, "init %d\n", rc); MPI_Abort(MPI_COMM_WORLD, 7); }
		if((rc = RK_MPI_SA_check_mem(&mem_dist))) { fprintf(stderr, "check_mem %d\n", rc); MPI_Abort(MPI_COMM_WORLD, 8); }
		rc = RK_MPI_SA_solve(final_time, &eqSystem);
		if(MPIprocs > 1) {
			/* every rank writes its own slab: <out>.<rank> */
			char name[4096];
			snprintf(name, sizeof(name), "%s.%d", argv[13], MPIrank);
			f = fopen(name, "wb");
		} else {
			f = fopen(argv[13], "wb");
		}
		fprintf(f, "%a %a %ld %ld %d\n", eqSystem.t, eqSystem.h, eqSystem.steps, eqSystem.steps_total, rc);
		for(q = 0; q < 3; q++)
			for(k = 0; k < n3; k++)
				for(j = 0; j < n2; j++)
					fwrite(solution + q * S + (long)(k + 2) * N1 * N2 + (long)(j + 2) * N1 + 2, sizeof(FLOAT), n1, f);
		fclose(f);
		RK_MPI_SA_cleanup();
	}
	FreePrecalcData();
	MPI_Finalize();
	return 0;
}
