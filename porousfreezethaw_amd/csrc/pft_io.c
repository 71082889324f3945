/*
 * pft_io.c -- NetCDF-classic snapshot datasets of the intertrack state (include/pft_io.h).
 *
 * The dataset is the one intertrack.c:2326-2548 writes through the NetCDF library (dimensions,
 * coordinate variables, u/p/gl, global attributes in the same order); this file writes and reads
 * the classic on-disk format directly (CDF-1, or CDF-2 when the 32-bit offsets would overflow),
 * so that no NetCDF installation is needed.  Every rank writes/reads only its own Z-slab planes
 * at their offsets in the shared file (pwrite/pread); no gather through the master.
 */
#define _XOPEN_SOURCE 700
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <unistd.h>

#include "../../include/pft_io.h"
#include "../../include/pft_comm.h"

/* classic-format tags */
enum { NC_DIMENSION = 10, NC_VARIABLE = 11, NC_ATTRIBUTE = 12 };
enum { NCT_CHAR = 2, NCT_INT = 4, NCT_DOUBLE = 6 };

/* attribute order of intertrack.c:2389 (param_info[], model.c:85-137) as pft_model.h indices */
static const struct { int idx; const char * name; } param_order[] = {
	{PFT_P_u_star, "u_star"}, {PFT_P_L, "L"},
	{PFT_P_water_cp, "water_cp"}, {PFT_P_ice_cp, "ice_cp"}, {PFT_P_glass_cp, "glass_cp"},
	{PFT_P_water_lambda, "water_lambda"}, {PFT_P_ice_lambda, "ice_lambda"}, {PFT_P_glass_lambda, "glass_lambda"},
	{PFT_P_water_rho, "water_rho"}, {PFT_P_ice_rho, "ice_rho"}, {PFT_P_glass_rho, "glass_rho"},
	{PFT_P_ball_radius, "ball_radius"}, {PFT_P_beads_scaling, "beads_scaling"},
	{PFT_P_beads_offset_x, "beads_offset_x"}, {PFT_P_beads_offset_y, "beads_offset_y"},
	{PFT_P_beads_offset_z, "beads_offset_z"}, {PFT_P_xi_gl, "xi_gl"}, {PFT_P_zeta, "zeta"},
	{PFT_P_xi, "xi"}, {PFT_P_a, "a"}, {PFT_P_b, "b"}, {PFT_P_alpha, "alpha"}, {PFT_P_mu, "mu"},
	{PFT_P_p_eps0, "p_eps0"}, {PFT_P_p_eps1, "p_eps1"}, {PFT_P_gamma, "gamma"},
	{PFT_P_top_temp1, "top_temp1"}, {PFT_P_top_temp2, "top_temp2"},
	{PFT_P_phase_switch_time, "phase_switch_time"}, {PFT_P_u_noise_amp, "u_noise_amp"},
};
#define NPARAM ((int)(sizeof(param_order) / sizeof(param_order[0])))
static const char * var_names[3] = {"u", "p", "gl"};     /* model.c:79-83 */

/* ---------------------------------------------------------------------------------------- */
/* big-endian encoding */

static uint64_t bswap64(uint64_t v) { return __builtin_bswap64(v); }
static uint64_t d2be(double d) { uint64_t u; memcpy(&u, &d, 8); return bswap64(u); }
static double be2d(uint64_t u) { double d; u = bswap64(u); memcpy(&d, &u, 8); return d; }

typedef struct { unsigned char * p; size_t n, cap; } buf_t;

static int bput(buf_t * b, const void * src, size_t n)
{
	if(b->n + n > b->cap) {
		size_t c = b->cap ? b->cap : 4096;
		unsigned char * q;
		while(c < b->n + n) c *= 2;
		if(!(q = (unsigned char *)realloc(b->p, c))) return -1;
		b->p = q; b->cap = c;
	}
	if(src) memcpy(b->p + b->n, src, n); else memset(b->p + b->n, 0, n);
	b->n += n;
	return 0;
}
static int put32(buf_t * b, uint32_t v) { v = __builtin_bswap32(v); return bput(b, &v, 4); }
static int put64(buf_t * b, uint64_t v) { v = bswap64(v); return bput(b, &v, 8); }
static int put_name(buf_t * b, const char * s)
{
	size_t n = strlen(s), pad = (4 - n % 4) % 4;
	return put32(b, (uint32_t)n) || bput(b, s, n) || bput(b, NULL, pad);
}
static int put_att_double(buf_t * b, const char * name, double v)
{
	uint64_t u = d2be(v);
	return put_name(b, name) || put32(b, NCT_DOUBLE) || put32(b, 1) || bput(b, &u, 8);
}
static int put_att_int(buf_t * b, const char * name, int v)
{
	return put_name(b, name) || put32(b, NCT_INT) || put32(b, 1) || put32(b, (uint32_t)v);
}
static int put_att_text(buf_t * b, const char * name, const char * s)
{
	size_t n = strlen(s), pad = (4 - n % 4) % 4;
	return put_name(b, name) || put32(b, NCT_CHAR) || put32(b, (uint32_t)n) || bput(b, s, n) || bput(b, NULL, pad);
}

/* ---------------------------------------------------------------------------------------- */
/* layout of the dataset: 3 coordinate variables, then u, p, gl */

typedef struct {
	int version;           /* 1 or 2 */
	long n1, n2, n3;
	uint64_t begin[6];     /* n3, n2, n1, u, p, gl */
	uint64_t vsize[6];
	uint64_t total;
} layout_t;

static int build_header(buf_t * b, layout_t * L, const pft_grid * g, const double * param,
                        const pft_snapshot_info * info, int pass)
{
	static const char * coord_names[3] = {"n3", "n2", "n1"};
	int q, rc = 0;
	b->n = 0;
	rc |= bput(b, "CDF", 3);
	{ unsigned char v = (unsigned char)L->version; rc |= bput(b, &v, 1); }
	rc |= put32(b, 0);                                          /* numrecs: no record dimension */
	/* dimensions (:2338-2340) */
	rc |= put32(b, NC_DIMENSION) || put32(b, 3);
	rc |= put_name(b, "n3") || put32(b, (uint32_t)L->n3);
	rc |= put_name(b, "n2") || put32(b, (uint32_t)L->n2);
	rc |= put_name(b, "n1") || put32(b, (uint32_t)L->n1);
	/* global attributes (:2382-2406) */
	rc |= put32(b, NC_ATTRIBUTE) || put32(b, (uint32_t)(3 + NPARAM + 8));
	rc |= put_att_double(b, "L1", g->L1) || put_att_double(b, "L2", g->L2) || put_att_double(b, "L3", g->L3);
	for(q = 0; q < NPARAM; q++) rc |= put_att_double(b, param_order[q].name, param[param_order[q].idx]);
	rc |= put_att_int(b, "calc_mode", info->calc_mode);
	rc |= put_att_double(b, "delta", info->delta) || put_att_double(b, "tau", info->tau);
	rc |= put_att_double(b, "t", info->t) || put_att_double(b, "final_time", info->final_time);
	rc |= put_att_int(b, "snapshot", info->snapshot) || put_att_int(b, "total_snapshots", info->total_snapshots);
	rc |= put_att_text(b, "title", info->title);
	/* variables (:2350-2354) */
	rc |= put32(b, NC_VARIABLE) || put32(b, 6);
	for(q = 0; q < 6; q++) {
		rc |= put_name(b, q < 3 ? coord_names[q] : var_names[q - 3]);
		if(q < 3) { rc |= put32(b, 1) || put32(b, (uint32_t)q); }
		else { rc |= put32(b, 3) || put32(b, 0) || put32(b, 1) || put32(b, 2); }
		rc |= put32(b, 0) || put32(b, 0);                       /* no variable attributes */
		rc |= put32(b, NCT_DOUBLE);
		rc |= put32(b, L->vsize[q] > 0xfffffffcULL ? 0xffffffffu : (uint32_t)L->vsize[q]);
		if(L->version == 1) rc |= put32(b, (uint32_t)L->begin[q]); else rc |= put64(b, L->begin[q]);
	}
	(void)pass;
	return rc ? -1 : 0;
}

static int make_layout(buf_t * b, layout_t * L, const pft_grid * g, const double * param,
                       const pft_snapshot_info * info, int version)
{
	int q;
	L->n1 = g->n1; L->n2 = g->n2; L->n3 = g->total_n3;
	L->vsize[0] = 8 * (uint64_t)L->n3; L->vsize[1] = 8 * (uint64_t)L->n2; L->vsize[2] = 8 * (uint64_t)L->n1;
	for(q = 3; q < 6; q++) L->vsize[q] = 8 * (uint64_t)L->n1 * L->n2 * L->n3;
	L->version = version ? version : 1;
	for(;;) {
		uint64_t off;
		memset(L->begin, 0, sizeof(L->begin));
		if(build_header(b, L, g, param, info, 0)) return -1;      /* header size with these widths */
		off = b->n;
		for(q = 0; q < 6; q++) { L->begin[q] = off; off += L->vsize[q]; }
		L->total = off;
		if(L->version == 1 && L->begin[5] > 0x7fffffffULL) {
			if(version == 1) return -2;                           /* does not fit CDF-1 */
			L->version = 2; continue;
		}
		break;
	}
	return build_header(b, L, g, param, info, 1);
}

/* ---------------------------------------------------------------------------------------- */

int pft_snapshot_title(char * buf, int size, const char * comment, double t)
{
	return snprintf(buf, (size_t)size, "Intertrack simulation (%s). Time: %g", comment ? comment : "", t) < 0 ? -2 : 0;
}

static int write_all(int fd, const void * p, size_t n, off_t off)
{
	const char * c = (const char *)p;
	while(n) {
		ssize_t w = pwrite(fd, c, n, off);
		if(w < 0) { if(errno == EINTR) continue; return -1; }
		c += w; n -= (size_t)w; off += w;
	}
	return 0;
}

static int read_all(int fd, void * p, size_t n, off_t off)
{
	char * c = (char *)p;
	while(n) {
		ssize_t r = pread(fd, c, n, off);
		if(r < 0) { if(errno == EINTR) continue; return -1; }
		if(r == 0) { errno = EIO; return -1; }
		c += r; n -= (size_t)r; off += r;
	}
	return 0;
}

int pft_snapshot_create(const char * path, const pft_grid * g, const double * param,
                        const pft_snapshot_info * info, int version)
{
	buf_t b = {0};
	layout_t L;
	int fd, rc = 0, q;
	long k;
	uint64_t * coord;
	if(!path || !g || !param || !info || version < 0 || version > 2) return -2;
	if(g->n1 < 1 || g->n2 < 1 || g->total_n3 < 1) return -2;
	if((rc = make_layout(&b, &L, g, param, info, version))) { free(b.p); return rc; }
	fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);           /* NC_CLOBBER */
	if(fd < 0) { free(b.p); return -1; }
	rc = write_all(fd, b.p, b.n, 0);
	/* coordinate variables, :2441-2443 (bcond_thickness_ = 0 in grid_IO_mode 1) */
	coord = (uint64_t *)malloc(8 * (size_t)(L.n3 > L.n2 ? (L.n3 > L.n1 ? L.n3 : L.n1) : (L.n2 > L.n1 ? L.n2 : L.n1)));
	if(!coord) rc = -1;
	for(q = 0; q < 3 && !rc; q++) {
		const long n = q == 0 ? L.n3 : q == 1 ? L.n2 : L.n1;
		const double Ld = q == 0 ? g->L3 : q == 1 ? g->L2 : g->L1;
		const double nd = (double)(q == 0 ? g->total_n3 : q == 1 ? g->n2 : g->n1);
		for(k = 0; k < n; k++) coord[k] = d2be(Ld * (0.5 + k - 0) / nd);
		rc = write_all(fd, coord, 8 * (size_t)n, (off_t)L.begin[q]);
	}
	free(coord);
	if(!rc && ftruncate(fd, (off_t)L.total)) rc = -1;              /* every slab's extent exists */
	if(close(fd) && !rc) rc = -1;
	free(b.p);
	return rc;
}

/* begin offsets of u, p, gl from a dataset's header (shared by read and write_slab) */
typedef struct {
	int version;
	long n1, n2, n3;
	uint64_t begin[3];
	pft_snapshot_info info;
	double param[PFT_PARAM_COUNT];
	int have_param[PFT_PARAM_COUNT];
} parsed_t;

typedef struct { const unsigned char * p; size_t n, at; int err; } rd_t;

static uint32_t get32(rd_t * r)
{
	uint32_t v;
	if(r->at + 4 > r->n) { r->err = 1; return 0; }
	memcpy(&v, r->p + r->at, 4); r->at += 4;
	return __builtin_bswap32(v);
}
static uint64_t get64(rd_t * r)
{
	uint64_t v;
	if(r->at + 8 > r->n) { r->err = 1; return 0; }
	memcpy(&v, r->p + r->at, 8); r->at += 8;
	return bswap64(v);
}
static void get_name(rd_t * r, char * out, size_t outsz)
{
	uint32_t n = get32(r);
	size_t pad = (4 - n % 4) % 4;
	if(r->err || r->at + n + pad > r->n) { r->err = 1; return; }
	if(out) { size_t c = n < outsz - 1 ? n : outsz - 1; memcpy(out, r->p + r->at, c); out[c] = 0; }
	r->at += n + pad;
}
static size_t type_size(uint32_t t) { return t == 1 || t == 2 ? 1 : t == 3 ? 2 : t == 4 || t == 5 ? 4 : t == 6 ? 8 : 0; }

static int parse_header(int fd, parsed_t * P)
{
	size_t cap = 1 << 16;
	unsigned char * p = NULL;
	rd_t r;
	uint32_t tag, n, q;
	long dims[8];
	int ndims = 0;
	memset(P, 0, sizeof(*P));
	for(;;) {                                                       /* read enough of the header */
		ssize_t got;
		unsigned char * np = (unsigned char *)realloc(p, cap);
		if(!np) { free(p); return -1; }
		p = np;
		got = pread(fd, p, cap, 0);
		if(got < 0) { free(p); return -1; }
		r.p = p; r.n = (size_t)got; r.at = 0; r.err = 0;
		if(got < 8 || memcmp(p, "CDF", 3) || (p[3] != 1 && p[3] != 2)) { free(p); return -3; }
		P->version = p[3];
		r.at = 4;
		(void)get32(&r);                                            /* numrecs */
		tag = get32(&r); n = get32(&r);                             /* dimensions */
		if(tag == NC_DIMENSION) for(q = 0; q < n && q < 8; q++) { get_name(&r, NULL, 0); dims[ndims++] = (long)get32(&r); }
		tag = get32(&r); n = get32(&r);                             /* global attributes */
		if(tag == NC_ATTRIBUTE) for(q = 0; q < n && !r.err; q++) {
			char name[64];
			uint32_t t, cnt;
			size_t sz, pad;
			int a;
			get_name(&r, name, sizeof(name));
			t = get32(&r); cnt = get32(&r);
			sz = type_size(t) * cnt; pad = (4 - sz % 4) % 4;
			if(r.err || r.at + sz + pad > r.n) { r.err = 1; break; }
			if(t == NCT_DOUBLE && cnt >= 1) {
				rd_t v = r;
				const uint64_t bits = get64(&v);                    /* already host order */
				double d;
				memcpy(&d, &bits, 8);
				if(!strcmp(name, "t")) P->info.t = d;
				else if(!strcmp(name, "L1")) P->info.L1 = d;
				else if(!strcmp(name, "L2")) P->info.L2 = d;
				else if(!strcmp(name, "L3")) P->info.L3 = d;
				else if(!strcmp(name, "tau")) P->info.tau = d;
				else if(!strcmp(name, "final_time")) P->info.final_time = d;
				else if(!strcmp(name, "delta")) P->info.delta = d;
				else for(a = 0; a < NPARAM; a++)
					if(!strcmp(name, param_order[a].name)) { P->param[param_order[a].idx] = d; P->have_param[param_order[a].idx] = 1; }
			} else if(t == NCT_INT && cnt >= 1) {
				rd_t v = r;
				const int i = (int)get32(&v);
				if(!strcmp(name, "snapshot")) P->info.snapshot = i;
				else if(!strcmp(name, "total_snapshots")) P->info.total_snapshots = i;
				else if(!strcmp(name, "calc_mode")) P->info.calc_mode = i;
			} else if(t == NCT_CHAR && !strcmp(name, "title")) {
				size_t c = cnt < sizeof(P->info.title) - 1 ? cnt : sizeof(P->info.title) - 1;
				memcpy(P->info.title, r.p + r.at, c); P->info.title[c] = 0;
			}
			r.at += sz + pad;
		}
		tag = get32(&r); n = get32(&r);                             /* variables */
		if(tag == NC_VARIABLE) for(q = 0; q < n && !r.err; q++) {
			char name[64];
			uint32_t nd, d, natt, a, t, sz;
			uint64_t begin;
			int vi;
			get_name(&r, name, sizeof(name));
			nd = get32(&r);
			for(d = 0; d < nd; d++) (void)get32(&r);
			if(get32(&r) == NC_ATTRIBUTE) {                          /* skip variable attributes */
				natt = get32(&r);
				for(a = 0; a < natt && !r.err; a++) {
					uint32_t cnt; size_t s2;
					get_name(&r, NULL, 0); t = get32(&r); cnt = get32(&r);
					s2 = type_size(t) * cnt; r.at += s2 + (4 - s2 % 4) % 4;
				}
			} else (void)get32(&r);
			t = get32(&r); sz = get32(&r);
			begin = P->version == 1 ? get32(&r) : get64(&r);
			(void)sz;
			for(vi = 0; vi < 3; vi++) if(!strcmp(name, var_names[vi]) && t == NCT_DOUBLE && nd == 3) P->begin[vi] = begin;
		}
		if(!r.err) break;
		if((size_t)got < cap) { free(p); return -3; }               /* truncated file */
		cap *= 4;                                                   /* header larger than the probe */
	}
	free(p);
	if(ndims < 3 || !P->begin[0] || !P->begin[1] || !P->begin[2]) return -3;
	P->n3 = dims[0]; P->n2 = dims[1]; P->n1 = dims[2];
	return 0;
}

int pft_snapshot_read_info(const char * path, int * n1, int * n2, int * total_n3,
                           pft_snapshot_info * info, double * param)
{
	parsed_t P;
	int fd, rc, q;
	if(!path) return -2;
	if((fd = open(path, O_RDONLY)) < 0) return -1;
	rc = parse_header(fd, &P);
	close(fd);
	if(rc) return rc;
	if(n1) *n1 = (int)P.n1;
	if(n2) *n2 = (int)P.n2;
	if(total_n3) *total_n3 = (int)P.n3;
	if(info) *info = P.info;
	if(param) for(q = 0; q < PFT_PARAM_COUNT; q++) if(P.have_param[q]) param[q] = P.param[q];
	return 0;
}

/* move this slab's interior planes between the host padded array and the dataset */
static int slab_io(const char * path, const pft_grid * g, double * x, int writing)
{
	parsed_t P;
	int fd, rc, q;
	long k, j, i;
	const long N1 = g->n1 + 2 * PFT_BCOND_THICKNESS, N2 = g->n2 + 2 * PFT_BCOND_THICKNESS;
	const long N3 = g->n3 + 2 * PFT_BCOND_THICKNESS, S = N1 * N2 * N3, plane = (long)g->n1 * g->n2;
	uint64_t * row;
	if(!path || !g || !x) return -2;
	if((fd = open(path, writing ? O_RDWR : O_RDONLY)) < 0) return -1;
	if((rc = parse_header(fd, &P))) { close(fd); return rc; }
	if(P.n1 != g->n1 || P.n2 != g->n2 || P.n3 != g->total_n3) { close(fd); return -4; }
	if(!(row = (uint64_t *)malloc(8 * (size_t)plane))) { close(fd); return -1; }
	for(q = 0; q < 3 && !rc; q++)
		for(k = 0; k < g->n3 && !rc; k++) {
			const off_t off = (off_t)(P.begin[q] + 8 * (uint64_t)((g->first_row + k) * plane));
			double * base = x + q * S + (k + PFT_BCOND_THICKNESS) * N1 * N2;
			if(writing) {
				for(j = 0; j < g->n2; j++)
					for(i = 0; i < g->n1; i++)
						row[j * g->n1 + i] = d2be(base[(j + PFT_BCOND_THICKNESS) * N1 + i + PFT_BCOND_THICKNESS]);
				rc = write_all(fd, row, 8 * (size_t)plane, off);
			} else {
				rc = read_all(fd, row, 8 * (size_t)plane, off);
				if(!rc) for(j = 0; j < g->n2; j++)
					for(i = 0; i < g->n1; i++)
						base[(j + PFT_BCOND_THICKNESS) * N1 + i + PFT_BCOND_THICKNESS] = be2d(row[j * g->n1 + i]);
			}
		}
	free(row);
	if(close(fd) && !rc) rc = -1;
	return rc;
}

int pft_snapshot_write_slab(const char * path, const pft_grid * g, const double * x)
{
	return slab_io(path, g, (double *)x, 1);
}

int pft_snapshot_read_slab(const char * path, const pft_grid * g, double * x)
{
	return slab_io(path, g, x, 0);
}

int pft_snapshot_write(const char * path, const pft_grid * g, const double * param,
                       const pft_snapshot_info * info, const double * x)
{
	pft_comm * c = pft_comm_current();
	long long err = 0;
	int rc = 0;
	if(!g) return -2;
	if(g->rank == 0) rc = pft_snapshot_create(path, g, param, info, 0);
	err = rc ? 1 : 0;
	pft_comm_allreduce_max_i64(c, &err);                           /* also the barrier */
	if(err) return rc ? rc : -1;
	rc = pft_snapshot_write_slab(path, g, x);
	err = rc ? 1 : 0;
	pft_comm_allreduce_max_i64(c, &err);
	return rc ? rc : (err ? -1 : 0);
}
