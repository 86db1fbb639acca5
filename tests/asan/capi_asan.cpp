// Host-side AddressSanitizer check of the C-ABI (SURVEY §5:
// "an ASan build of the C-ABI host code").  Linked against
// libartsbir_hip_asan.so, whose host code is compiled with
// -Xarch_host -fsanitize=address (device code untouched); runs on a machine
// without a GPU: every call below returns before any kernel launch or device
// allocation — the autotune table parser and writer, the error-message buffer
// with over-long arguments, and the argument checks of the entry points.
// Prints "asan capi ok" and exits 0; ASan aborts on any invalid access.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/artsbir.h"

static int fails = 0;
#define EXPECT(c)                                                 \
  do {                                                            \
    if (!(c)) { fprintf(stderr, "FAILED: %s (line %d)\n", #c, __LINE__); ++fails; } \
  } while (0)

static void write_file(const char* path, const char* text) {
  FILE* f = fopen(path, "w");
  if (!f) { perror(path); exit(2); }
  fputs(text, f);
  fclose(f);
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  char path[4096];
  EXPECT(artsbir_version() == 1);

  // the error buffer: a path far longer than the 512-byte message buffer
  char longpath[3000];
  memset(longpath, 'x', sizeof(longpath) - 1);
  longpath[0] = '/';
  longpath[sizeof(longpath) - 1] = 0;
  EXPECT(artsbir_tune_load(longpath) == -1);
  EXPECT(strlen(artsbir_last_error()) < 512 && strncmp(artsbir_last_error(), "tune_load: cannot open", 22) == 0);

  // autotune table: two valid lines, then a truncated one (parsing stops there)
  snprintf(path, sizeof(path), "%s/asan_tune_a.txt", dir);
  write_file(path,
             "c 1152 56 56 64 64 3 3 1 1 56 56 0 1 3 0 22\n"
             "w 3612672 56 56 64 256 1 1 1 0 1 64 256 64 101\n"
             "c 12 3 4\n");
  EXPECT(artsbir_tune_load(path) == 2);
  // retired candidates are skipped (not counted); an over-long token stops the
  // parser without reading past its 3-character tag buffer
  snprintf(path, sizeof(path), "%s/asan_tune_b.txt", dir);
  {
    char big[9000];
    memset(big, 'c', sizeof(big) - 1);
    big[sizeof(big) - 1] = 0;
    char text[9200];
    snprintf(text, sizeof(text), "c 1 1 1 32 32 1 1 1 0 1 1 0 0 1 0 23\nw 1 1 1 8 8 1 1 1 0 1 8 8 8 -3\n%s 1 2\n", big);
    write_file(path, text);
  }
  EXPECT(artsbir_tune_load(path) == 0);
  snprintf(path, sizeof(path), "%s/asan_tune_c.txt", dir);
  write_file(path, "");
  EXPECT(artsbir_tune_load(path) == 0);
  snprintf(path, sizeof(path), "%s/asan_tune_out.txt", dir);
  EXPECT(artsbir_tune_save(path) == 0);
  EXPECT(artsbir_tune_load(path) >= 2);

  // argument checks that return before touching the device
  EXPECT(artsbir_gemm_tn(ARTSBIR_DT_BF16, 16, 7, 8, NULL, 8, NULL, 8, NULL, NULL) == -1);
  EXPECT(strstr(artsbir_last_error(), "gemm_tn") != NULL);
  EXPECT(artsbir_gemm_nt_fp8(256, 256, 100, NULL, NULL, NULL, NULL, NULL, NULL, ARTSBIR_DT_BF16, 0, NULL) == -1);
  EXPECT(artsbir_quantize_fp8(ARTSBIR_DT_BF16, NULL, 0, NULL, NULL, NULL) == -1);
  EXPECT(artsbir_mha_bwd(ARTSBIR_DT_BF16, NULL, NULL, NULL, NULL, 300, 1, 1, NULL, NULL, NULL, NULL) == -1);
  EXPECT(artsbir_stream_create_cu_mask(NULL, 0, NULL) == -1);

  if (fails) return 1;
  printf("asan capi ok\n");
  return 0;
}
