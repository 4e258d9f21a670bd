/* vmqg_set_option("reader_records") when the two reader copies of the record
 * table cannot be allocated: the call answers VMQG_E_NOMEM — no
 * exception crosses the C ABI — and leaves the context as it was, so the
 * option can be turned on once memory is there.  The address-space limit is
 * set just above the process's current size, below what the copies need. */
#include <stdio.h>
#include <string.h>
#include <unistd.h>
#include <sys/resource.h>
#include "vmqg.h"

static long vm_bytes(void) {
  long pages = 0;
  FILE* f = fopen("/proc/self/statm", "r");
  if (!f || fscanf(f, "%ld", &pages) != 1) pages = 0;
  if (f) fclose(f);
  return pages * sysconf(_SC_PAGESIZE);
}

int main(void) {
  vmqg_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = -1;
  cfg.hint_records = 1u << 23;   /* a 128-MB record region: the copies need 256 MB */
  int err = 0;
  vmqg_ctx* ctx = vmqg_create(&cfg, &err);
  if (!ctx || err) { printf("create %d\n", err); return 1; }
  struct rlimit old, lim;
  getrlimit(RLIMIT_AS, &old);
  lim = old;
  lim.rlim_cur = (rlim_t)vm_bytes() + (64u << 20);
  if (setrlimit(RLIMIT_AS, &lim)) { printf("setrlimit\n"); return 2; }
  const int rc = vmqg_set_option(ctx, "reader_records", 1);
  setrlimit(RLIMIT_AS, &old);
  if (rc != VMQG_E_NOMEM) { printf("limited: %d\n", rc); return 3; }
  vmqg_stats_t st;
  if (vmqg_stats(ctx, &st) != VMQG_OK) { printf("stats\n"); return 4; }
  const int rc2 = vmqg_set_option(ctx, "reader_records", 1);
  if (rc2 != VMQG_OK) { printf("unlimited: %d\n", rc2); return 5; }
  vmqg_destroy(ctx);
  printf("ok\n");
  return 0;
}
