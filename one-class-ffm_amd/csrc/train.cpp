// train.cpp — drop-in replacement for the reference's `train` binary
// (train.cpp:1-208): same argv grammar, defaults, stdout table, model file
// and exit codes, running the epoch on the GPU through the C ABI.
//
//   train [options] item_file train_file
//   -l lambda  -t iters  -p test_file  -o model_file  -w omega  -r rating
//   -c threads  -k rank  --ns  --freq
// Build-only options (the reference would take them for the item file):
//   --fp32 / --fp64 (default fp64, the reference's arithmetic type),
//   --device N.
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>

#include "../../include/ocffm.h"

static std::string usage() {
  return "usage: train [options] item_feature_file train_file\n"
         "\n"
         "options:\n"
         "-l <lambda_2>: set regularization coefficient on r regularizer (default 1e-5)\n"
         "-t <iter>: set number of iterations (default 20)\n"
         "-p <path>: set path to test set\n"
         "-o <path>: set path to save model file\n"
         "-w <omega>: set cost weight for the negatives (default 0.1)\n"
         "-r <rating>: set rating for the negatives (default -1)\n"
         "-c <threads>: set number of cores\n"
         "-k <rank>: set number of rank (default 4)\n"
         "--ns: no self-side field pairs\n"
         "--freq: enable freq-aware lambda\n"
         "--fp32 | --fp64: device arithmetic (default fp64)\n"
         "--device <n>: HIP device ordinal\n";
}

// train.cpp:22-32: at least one digit somewhere in the token.
static bool is_numerical(const char *s) {
  for (; *s; s++)
    if (std::isdigit((unsigned char)*s)) return true;
  return false;
}

struct Fail : std::runtime_error {
  int code;
  Fail(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

static void check(int st) {
  if (st != OCFFM_OK) throw Fail(st, ocffm_last_error());
}

int main(int argc, char **argv) {
  ocffm_param prm;
  ocffm_param_default(&prm);
  std::string te_path, model_path;
  try {
    if (argc == 1) throw std::invalid_argument(usage());
    int i = 1;
    for (; i < argc; i++) {
      const std::string a = argv[i];
      auto value = [&](bool numeric, const char *msg) -> const char * {
        if (i + 1 >= argc) throw std::invalid_argument(msg);
        i++;
        if (numeric && !is_numerical(argv[i])) throw std::invalid_argument(a + " should be followed by a number");
        return argv[i];
      };
      if (a == "-l") prm.lambda = std::atof(value(true, "need to specify l regularization coefficient after -l"));
      else if (a == "-k") prm.k = (uint32_t)std::atoi(value(true, "need to specify rank after -k"));
      else if (a == "-t") prm.nr_pass = (uint32_t)std::atoi(value(true, "need to specify max number of iterations after -t"));
      else if (a == "-w") prm.omega = std::atof(value(true, "need to specify omega after -w"));
      else if (a == "-r") prm.r = std::atof(value(true, "need to specify rating after -r"));
      else if (a == "-c") prm.nr_threads = (uint32_t)std::atof(value(true, "missing core numbers after -c"));
      else if (a == "-p") te_path = value(false, "need to specify path after -p");
      else if (a == "-o") model_path = value(false, "need to specify path after -o");
      else if (a == "--ns") prm.self_side = 0;
      else if (a == "--freq") prm.freq = 1;
      else if (a == "--fp32") prm.precision = OCFFM_FP32;
      else if (a == "--fp64") prm.precision = OCFFM_FP64;
      else if (a == "--device") prm.device = std::atoi(value(true, "need a device ordinal after --device"));
      else break;
    }
    if (i >= argc) throw std::invalid_argument("training data not specified");
    if (i + 1 >= argc) throw std::invalid_argument("training data not specified");
    const std::string item_path = argv[i], tr_path = argv[i + 1];

    // train.cpp:177-196.  OCFFM_TIMING=1: phase wall times on stderr.
    const bool timing = std::getenv("OCFFM_TIMING") != nullptr;
    auto t_prev = std::chrono::steady_clock::now();
    auto phase = [&](const char *name) {
      const auto t = std::chrono::steady_clock::now();
      if (timing) std::fprintf(stderr, "[timing] %-8s %9.3f ms\n", name, std::chrono::duration<double, std::milli>(t - t_prev).count());
      t_prev = t;
    };
    ocffm_data *U = nullptr, *V = nullptr, *Ut = nullptr;
    check(ocffm_data_read(tr_path.c_str(), 1, nullptr, 0, &U));
    check(ocffm_data_read(item_path.c_str(), 0, nullptr, 0, &V));
    check(ocffm_data_trans_y(V, U));
    if (!te_path.empty()) {
      ocffm_data_info info;
      check(ocffm_data_get_info(U, &info));
      std::uint64_t *ds = new std::uint64_t[info.f ? info.f : 1];
      check(ocffm_data_get_ds(U, ds));
      check(ocffm_data_read(te_path.c_str(), 1, ds, (uint32_t)info.f, &Ut));
      delete[] ds;
    }
    phase("read");
    ocffm_problem *prob = nullptr;
    check(ocffm_problem_create(U, Ut, V, &prm, &prob));
    phase("create");
    // The reference's init is the first consumer of the process rand()
    // stream (implicit seed 1, ffm.cpp:72); HIP/RCCL start-up above may have
    // drawn from it, so restore that state before the draws.
    std::srand(1);
    check(ocffm_problem_init(prob));
    check(ocffm_problem_sync(prob));
    phase("init");
    check(ocffm_problem_solve(prob));
    phase("solve");
    if (!model_path.empty()) check(ocffm_problem_save_model(prob, model_path.c_str()));
    phase("save");
    ocffm_problem_destroy(prob);
    ocffm_data_free(U);
    ocffm_data_free(V);
    if (Ut) ocffm_data_free(Ut);
  } catch (std::invalid_argument &e) {
    std::cerr << e.what() << std::endl;
    return 1;
  } catch (Fail &e) {
    std::cerr << "error: " << e.what() << std::endl;
    return e.code == OCFFM_E_ARG ? 1 : 2;
  }
  return 0;
}
