// The host runtime's worker pool under ThreadSanitizer (CPU only, no GPU):
// lsbm_test_pool_stress (every piece of every job runs exactly once, with
// nested jobs and more callers than job slots) built together with
// host_session.cc, host_numa.cc and status.cc with -fsanitize=thread; the
// engine entry points a session would need are stubbed (no session is made).
#include <stdio.h>

extern "C" int lsbm_test_pool_stress(int callers, int jobs, int max_pieces);
extern "C" int lsbm_host_threads(void);
extern "C" int lsbm_crc32c_init(int) { return -1; }
extern "C" const char* lsbm_crc32c_last_error(void) { return "stub"; }

int main() {
  const int threads = lsbm_host_threads();
  int bad = 0;
  for (int i = 0; i < 5; i++) bad += lsbm_test_pool_stress(8, 200, 64) + lsbm_test_pool_stress(70, 5, 8);
  printf("%s threads=%d bad=%d\n", bad ? "FAILED" : "OK", threads, bad);
  return bad != 0;
}
