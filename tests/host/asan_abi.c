/* Host-side checks of the C ABI under AddressSanitizer + UBSan (SURVEY 5 "race detection /
 * sanitizers": host code only -- GPU sanitizers are not available on this pool).
 * Built and run by tests/test_host_asan.py against libhdgnn built with
 * -Xarch_host -fsanitize=address,undefined; needs no GPU: it drives every entry point's
 * argument validation, sizing and error reporting, and the device entry points up to the
 * point where they would need a device (they must fail cleanly, never touch memory). */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "hdgnn.h"

static int fails = 0;
#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      fprintf(stderr, "FAIL %s:%d: %s (last error: %s)\n", __FILE__, __LINE__, #c, \
              hdg_last_error());                                                  \
      ++fails;                                                                    \
    }                                                                             \
  } while (0)

static hdg_shape shape(int b, int ne, int nc, int v, int path) {
  hdg_shape s;
  memset(&s, 0, sizeof s);
  s.batch = b;
  s.ne = ne;
  s.nc = nc;
  s.variant = v;
  s.batch_global = b;
  s.path = path;
  s.flags = 0;
  return s;
}

int main(void) {
  CHECK(hdg_version() == HDG_ABI_VERSION);
  for (int v = 1; v <= 4; ++v) {
    CHECK(hdg_param_count(v) > 0);
    CHECK(hdg_grad_len(v) > hdg_param_count(v));
  }
  CHECK(hdg_param_count(0) < 0 && strlen(hdg_last_error()) > 0);
  CHECK(hdg_param_count(5) < 0);
  const int shapes[][3] = {{100, 200, 74}, {2, 250, 150}, {1, 256, 160}, {1, 1024, 512},
                           {1, 4096, 40}, {1, 40, 2048}, {3, 7, 5}, {1, 2, 2}};
  for (unsigned i = 0; i < sizeof shapes / sizeof shapes[0]; ++i) {
    for (int v = 1; v <= 4; ++v) {
      for (int path = 0; path <= 2; ++path) {
        hdg_shape s = shape(shapes[i][0], shapes[i][1], shapes[i][2], v, path);
        const int r = hdg_resolve_path(&s);
        if (r < 0) continue;                       /* shape beyond this path: error set */
        s.path = r;
        CHECK(hdg_workspace_bytes(&s) > 0);
        CHECK(hdg_prep_bytes(&s) > 0);
        int64_t st = 0, ks = 0, kt = 0, nc = 0;
        if (hdg_prep_counts_layout(&s, &st, &ks, &kt, &nc) == 0)
          CHECK(st > 0 && ks >= 0 && kt > ks && nc > kt);
      }
    }
  }
  hdg_shape bad = shape(1, 5000, 74, 2, 0);          /* beyond every path */
  CHECK(hdg_resolve_path(&bad) < 0);
  bad = shape(0, 200, 74, 2, 0);
  CHECK(hdg_resolve_path(&bad) < 0);
  bad = shape(1, 200, 74, 9, 0);
  CHECK(hdg_resolve_path(&bad) < 0);
  CHECK(hdg_resolve_path(NULL) < 0);
  CHECK(hdg_workspace_bytes(NULL) == 0);
  CHECK(hdg_prep_bytes(NULL) == 0);
  CHECK(hdg_dp_mailbox_bytes() > 0);
  /* device entry points with missing pointers: argument errors, no memory touched */
  hdg_shape s = shape(2, 200, 74, 2, 0);
  hdg_batch bt;
  memset(&bt, 0, sizeof bt);
  hdg_state stt;
  memset(&stt, 0, sizeof stt);
  hdg_outputs out;
  memset(&out, 0, sizeof out);
  CHECK(hdg_prepare(&s, NULL, NULL) != 0);
  CHECK(hdg_prepare(NULL, &bt, NULL) != 0);
  CHECK(hdg_fwd_bwd(&s, NULL, NULL, NULL, NULL, NULL, NULL) != 0);
  CHECK(hdg_train_step(&s, &bt, NULL, 3e-4f, &out, NULL, NULL, NULL) != 0);
  CHECK(hdg_forward(&s, &bt, NULL, &out, NULL, NULL, NULL) != 0);
  CHECK(hdg_adam_tf(&s, NULL, NULL, 3e-4f, NULL, NULL) != 0);
  CHECK(hdg_pack_classes(NULL, 2, 200, NULL, NULL) != 0);
  CHECK(hdg_dp_allreduce(NULL, NULL, NULL, 0, NULL, NULL) != 0);
  CHECK(strlen(hdg_last_error()) > 0);
  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("asan_abi: all checks passed\n");
  return 0;
}
