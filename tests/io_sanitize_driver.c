/* Host sanitizer driver for csrc/cloudsc_io.c (tests/test_io.py::
 * test_io_readers_under_address_sanitizer): every reader, on each directory
 * or HDF5 file named on the command line, followed by cloudsc_io_free on
 * success.  Built with -fsanitize=address,undefined (leak checking on), so an
 * out-of-bounds access, undefined behaviour or a leak on a success or error
 * path fails the run.  Prints one return code per (argument, reader). */
#include <stdio.h>
#include <string.h>

#include "cloudsc_io.h"

int main(int argc, char **argv) {
  for (int i = 1; i < argc; i++) {
    const char *a = argv[i];
    const size_t n = strlen(a);
    if (n > 3 && strcmp(a + n - 3, ".h5") == 0) {
      cloudsc_dataset_t d;
      memset(&d, 0, sizeof(d));
      int rc = cloudsc_io_load_hdf5(a, NULL, &d);
      if (rc == 0) cloudsc_io_free(&d);
      printf("%d\n", rc);
      continue;
    }
    int (*readers[3])(const char *, int, cloudsc_dataset_t *) = {cloudsc_io_load_serialbox, cloudsc_io_load_raw,
                                                                 cloudsc_io_load_dir};
    for (int r = 0; r < 3; r++) {
      cloudsc_dataset_t d;
      memset(&d, 0, sizeof(d));
      int rc = readers[r](a, 1, &d);
      if (rc == 0) cloudsc_io_free(&d);
      printf("%d ", rc);
    }
    printf("\n");
  }
  return 0;
}
