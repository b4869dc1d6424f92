// dev_probe.c -- one process start as the NF makes it, reduced to the device
// part: count the devices through libxsknf_gpu, create and destroy a launched
// host-path context on device 0 (its streams, events and pinned arrays), exit.
// Prints one JSON line; on failure the library's error text says what the
// process saw (xsknf_gpu_device_count: HIP's error, /dev/kfd and render-node
// access, *_VISIBLE_DEVICES, the KFD processes).  Driven by
// tools/nf_start_probe.py, which starts it back to back from a process that
// never touched the GPU while its parent holds a GPU context (the GPU suite's
// shape: tests/test_gpu_app.py).  `dev_probe [hold_s]` keeps the context hold_s
// seconds before destroying it.  Measurement infra, not the product.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "xsknf_gpu.h"

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
	const double hold = argc > 1 ? atof(argv[1]) : 0.0;   // seconds to keep the context
	const double t0 = now_s();
	int count = 0;
	int rc = xsknf_gpu_device_count(&count);
	const double t1 = now_s();
	if (rc) {
		printf("{\"pid\": %d, \"ok\": false, \"stage\": \"device_count\", \"rc\": %d, \"init_s\": %.3f, "
		       "\"error\": \"%s\"}\n", (int)getpid(), rc, t1 - t0, xsknf_gpu_last_error());
		return 1;
	}
	struct xsknf_gpu_ctx *ctx = NULL;
	rc = xsknf_gpu_ctx_create(&ctx, 0, XSKNF_GPU_PATH_ZEROCOPY, 64, 64);
	if (!rc && hold > 0)
		usleep((useconds_t)(hold * 1e6));
	if (!rc)
		rc = xsknf_gpu_ctx_destroy(ctx);
	const double t2 = now_s();
	printf("{\"pid\": %d, \"ok\": %s, \"stage\": \"ctx\", \"rc\": %d, \"devices\": %d, \"init_s\": %.3f, "
	       "\"ctx_s\": %.3f, \"error\": \"%s\"}\n", (int)getpid(), rc ? "false" : "true", rc, count, t1 - t0,
	       t2 - t1, rc ? xsknf_gpu_last_error() : "");
	return rc ? 1 : 0;
}
