#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
static void attr(const char *tag, void *p) {
  hipPointerAttribute_t a{};
  hipError_t e = hipPointerGetAttributes(&a, p);
  unsigned f = 0;
  hipError_t e2 = hipHostGetFlags(&f, p);
  printf("%s: attr rc=%d type=%d | getflags rc=%d flags=%u\n", tag, (int)e, (int)a.type, (int)e2, f);
  (void)hipGetLastError();
}
int main() {
  size_t n = 64 << 20;
  char *p = (char *)aligned_alloc(4096, n);
  for (size_t i = 0; i < n; i += 4096) p[i] = 1;
  attr("pageable", p);
  printf("reg1 %d\n", (int)hipHostRegister(p, n, hipHostRegisterPortable));
  attr("registered", p);
  attr("registered+4096", p + 4096);
  printf("reg2 %d\n", (int)hipHostRegister(p, n, hipHostRegisterPortable));
  (void)hipGetLastError();
  printf("unreg1 %d\n", (int)hipHostUnregister(p));
  (void)hipGetLastError();
  attr("after unreg1", p);
  printf("unreg2 %d\n", (int)hipHostUnregister(p));
  (void)hipGetLastError();
  attr("after unreg2", p);
  return 0;
}
