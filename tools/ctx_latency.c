// ctx_latency.c -- where a small host-path batch's time goes: CPU time inside
// xsknf_gpu_ctx_submit (descriptor copy, launch or doorbell) and inside
// xsknf_gpu_ctx_wait, for batches of N frames of LEN bytes in a pinned UMEM,
// DEPTH - 1 batches in flight behind the one being submitted (default 2, at most 8; 1 =
// each batch waited for right after its submit: the round trip itself).
// WORKERS (default 1) threads run the same loop at once, each with its own
// context and UMEM, as the AF_XDP workers of src/xsknf.c:1075-1095 would (on
// RESIDENT they share the device's one resident kernel).  The path may be a
// comma-separated list, dealt to the workers in turn (RESIDENT,ZEROCOPY: a mixed
// set, the resident kernel's hardware queue beside the launches' streams); the
// output then also has each path's mean per batch.
//   ctx_latency LEN N ITERS [ZEROCOPY|STAGED|RESIDENT[,...] [DEPTH [WORKERS]]]
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/xsknf_gpu.h"

static double now_us(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

struct worker {
	unsigned len, n, iters, depth;
	int path;
	pthread_barrier_t *start;
	int rc;
	double us_per_batch, submit_us, wait_us;
};

static void *run(void *p)
{
	struct worker *w = p;
	const unsigned n = w->n, len = w->len;
	const unsigned nb = 64;   // distinct batches cycled through
	const size_t chunk = 2048, size = (size_t)nb * n * chunk;
	uint8_t *umem = aligned_alloc(4096, size);
	struct xsknf_gpu_desc *d = malloc(sizeof(*d) * (size_t)nb * n);
	int32_t *v = malloc(sizeof(int32_t) * (size_t)nb * n);
	struct xsknf_gpu_ctx *c = NULL;
	w->rc = 1;
	if (!umem || !d || !v)
		goto out;
	memset(umem, 0x5a, size);
	for (size_t i = 0; i < (size_t)nb * n; i++) {
		uint8_t *f = umem + i * chunk + 256;
		f[12] = 8, f[13] = 0, f[14] = 0x45, f[23] = 17;
		d[i].addr = i * chunk + 256;
		d[i].len = len;
		d[i].options = 0;
	}
	const struct xsknf_csum_opts o = {1, XSKNF_CSUM_ACTION_REDIRECT, 1, 0};
	if (xsknf_gpu_ctx_create(&c, 0, w->path, n, len) || xsknf_gpu_ctx_register_umem(c, umem, size)) {
		fprintf(stderr, "ctx: %s\n", xsknf_gpu_last_error());
		pthread_barrier_wait(w->start);
		goto out;
	}
	pthread_barrier_wait(w->start);
	double t_sub = 0, t_wait = 0;
	uint64_t tk[8] = {0};
	const double t0 = now_us();
	for (unsigned i = 0; i < w->iters; i++) {
		const unsigned b = i % nb;
		double a = now_us();
		if (xsknf_gpu_ctx_submit(c, d + (size_t)b * n, n, 0, &o, v + (size_t)b * n, &tk[i % 8]))
			goto out;
		double m = now_us();
		if (i + 1 >= w->depth && xsknf_gpu_ctx_wait(c, tk[(i + 1 - w->depth) % 8]))
			goto out;
		double e = now_us();
		if (i >= 16) {
			t_sub += m - a;
			t_wait += e - m;
		}
	}
	if (xsknf_gpu_ctx_wait(c, tk[(w->iters - 1) % 8]))
		goto out;
	const unsigned k = w->iters - 16;
	w->us_per_batch = (now_us() - t0) / w->iters;
	w->submit_us = t_sub / k;
	w->wait_us = t_wait / k;
	w->rc = 0;
out:
	if (c)
		xsknf_gpu_ctx_destroy(c);
	free(umem);
	free(d);
	free(v);
	return NULL;
}

int main(int argc, char **argv)
{
	if (argc < 4)
		return 2;
	struct worker proto = {0};
	proto.len = (unsigned)atoi(argv[1]);
	proto.n = (unsigned)atoi(argv[2]);
	proto.iters = (unsigned)atoi(argv[3]);
	int paths[8], npaths = 0;
	char spec[128];
	snprintf(spec, sizeof(spec), "%s", argc > 4 ? argv[4] : "ZEROCOPY");
	for (char *t = strtok(spec, ","); t && npaths < 8; t = strtok(NULL, ","))
		paths[npaths++] = !strcmp(t, "STAGED") ? XSKNF_GPU_PATH_STAGED
		                  : !strcmp(t, "RESIDENT") ? XSKNF_GPU_PATH_RESIDENT
		                                           : XSKNF_GPU_PATH_ZEROCOPY;
	if (npaths == 0)
		return 2;
	proto.path = paths[0];
	proto.depth = argc > 5 ? (unsigned)atoi(argv[5]) : 2;
	const unsigned workers = argc > 6 ? (unsigned)atoi(argv[6]) : 1;
	if (proto.depth < 1 || proto.depth > 8 || proto.iters <= 16 || workers < 1 || workers > 64)
		return 2;
	pthread_barrier_t start;
	pthread_barrier_init(&start, NULL, workers);
	struct worker w[64];
	pthread_t tid[64];
	for (unsigned i = 0; i < workers; i++) {
		w[i] = proto;
		w[i].path = paths[i % npaths];
		w[i].start = &start;
		if (pthread_create(&tid[i], NULL, run, &w[i]))
			return 1;
	}
	double per = 0, sub = 0, wait = 0, worst = 0, path_us[3] = {0}, mpps = 0;
	unsigned path_n[3] = {0};
	int rc = 0;
	for (unsigned i = 0; i < workers; i++) {
		pthread_join(tid[i], NULL);
		rc |= w[i].rc;
		path_us[w[i].path] += w[i].us_per_batch;
		path_n[w[i].path]++;
		if (w[i].us_per_batch > 0)
			mpps += proto.n / w[i].us_per_batch;
		per += w[i].us_per_batch / workers;
		sub += w[i].submit_us / workers;
		wait += w[i].wait_us / workers;
		if (w[i].us_per_batch > worst)
			worst = w[i].us_per_batch;
	}
	if (rc) {
		fprintf(stderr, "ctx_latency: a worker failed: %s\n", xsknf_gpu_last_error());
		return 1;
	}
	static const char *const names[3] = {"ZEROCOPY", "STAGED", "RESIDENT"};
	printf("{\"len\": %u, \"n\": %u, \"path\": \"%s\", \"depth\": %u, \"workers\": %u, \"us_per_batch\": %.2f, "
	       "\"us_per_batch_worst_worker\": %.2f, \"submit_cpu_us\": %.2f, \"wait_us\": %.2f, "
	       "\"mpps_all_workers\": %.2f", proto.len, proto.n, argc > 4 ? argv[4] : "ZEROCOPY", proto.depth, workers, per,
	       worst, sub, wait, npaths > 1 ? mpps : workers * proto.n / per);
	if (npaths > 1) {
		printf(", \"us_per_batch_by_path\": {");
		for (int p = 0, first = 1; p < 3; p++)
			if (path_n[p]) {
				printf("%s\"%s\": %.2f", first ? "" : ", ", names[p], path_us[p] / path_n[p]);
				first = 0;
			}
		printf("}");
	}
	printf("}\n");
	return 0;
}
