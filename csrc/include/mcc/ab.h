// A/B switches of the engine and the kernels, all behind ONE environment
// variable:  MCC_AB="name[=value],name[=value],..."  (e.g. MCC_AB=no_lenet or
// MCC_AB=igemm_tile=128,side_stream).  The defaults are the measured winners;
// every switch selects an older or measured-slower path for comparison runs
// and each has an A/B record in profiles/ (docs/ARCHITECTURE.md §6 lists
// them).  Read at plan time (GpuNet construction) or launch time, never
// cached, so a test can flip a switch between two nets.
#pragma once

#include <cstdlib>
#include <cstring>

namespace mcc {

// Value of `name` in MCC_AB: the integer after '=' if given, 1 if the name
// appears bare, `dflt` if absent.
inline int ab_int(const char* name, int dflt) {
  const char* s = std::getenv("MCC_AB");
  if (!s) return dflt;
  const size_t n = std::strlen(name);
  while (*s) {
    while (*s == ',' || *s == ' ') ++s;
    const char* e = s;
    while (*e && *e != ',') ++e;
    if ((size_t)(e - s) >= n && std::strncmp(s, name, n) == 0 && (s + n == e || s[n] == '='))
      return s + n == e ? 1 : std::atoi(s + n + 1);
    s = e;
  }
  return dflt;
}
inline bool ab_flag(const char* name) { return ab_int(name, 0) != 0; }

}  // namespace mcc
