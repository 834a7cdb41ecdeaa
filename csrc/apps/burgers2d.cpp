// Native burgers2d executable (reference CLI; see csrc/runtime/app.cpp).
#include <cstdio>
#include <exception>

#include "runtime.hpp"

namespace advdiff::rt {
int run_app(int argc, char** argv, Physics phys, int dims);
}

int main(int argc, char** argv) {
  try {
    return advdiff::rt::run_app(argc, argv, advdiff::rt::Physics::Burgers, 2);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "burgers2d: %s\n", e.what());
    return 1;
  }
}
