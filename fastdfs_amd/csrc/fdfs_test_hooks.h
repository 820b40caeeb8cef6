/* Test hooks of libfdfs_gpu: compiled only into the test build
 * (`make test-hooks` -> fastdfs_amd/lib/test/libfdfs_gpu.so, fdfs_api.cpp
 * with FDFS_TEST_HOOKS), never into the shipped library or include/. */
#ifndef FDFS_TEST_HOOKS_H
#define FDFS_TEST_HOOKS_H

#include "../../include/fdfs_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fault injection for tests of the error path: queues on `stream` what a
 * signature launch whose size binning went wrong leaves behind (the lane
 * path's error count raised by one), so that a later call of the context --
 * the first whose entry check sees it, whatever calls were queued in between
 * on any stream -- returns EIO once. */
int fdfs_gpu_inject_error(fdfs_gpu_ctx *ctx, void *stream);

#ifdef __cplusplus
}
#endif
#endif
