// Shared driver of the native executables (bin/diffusion2d, diffusion3d, burgers2d,
// burgers3d) with the reference's positional command lines:
//
//   diffusion2d  K L W Nx Ny iters [bx by]           (MultiGPU/Diffusion2d_Baseline/main.c:36-51)
//   diffusion3d  K L W H Nx Ny Nz iters [bx by bz]   (MultiGPU/Diffusion3d_Baseline/main.c:36-54)
//   burgers2d    tEnd CFL L W Nx Ny [bx by]          (MultiGPU/Burgers2d_Baseline/main.c:36-51)
//   burgers3d    tEnd CFL L W H Nx Ny Nz [bx by bz]  (MultiGPU/Burgers3d_Baseline/main.c:36-54)
//
// plus named options (runtime replacements of the reference's #defines, §2.7):
//   --ic NAME  --order 2|4  --safety S  --weno js|z|js7  --visc C  --fp32  --no-overlap
//   --[no-]boundary-on-comm (overlap: the boundary launch on the comm stream; default on
//   for --transport rccl and ipc; ADVDIFF_BCOMM=0/1)
//   --fused-put (--transport ipc slabs: the step / stage launch stores its boundary planes
//   into the neighbours' ghost planes itself; ADVDIFF_FUSED_PUT=0/1)
//   --integrator ssprk3|lsrk45  --no-fused  --transport rccl|ipc|socket  --write FILE
//   --write-ghosts FILE (the reference's multi-GPU result.bin: every rank's slab WITH its
//   ghost planes, MultiGPU/Diffusion3d_Baseline/main.c:341)  --error-norms
//   --decomp slab|PZxPYxPX|PYxPX (process grid in array order: Cartesian blocks, cart.cpp;
//   default z-slabs as the reference)  --geometry (print every rank's launch / halo
//   geometry as JSON lines and exit; no GPU work)  --graph / --no-graph (hipGraph
//   stepping, Engine::steps; default: on for the single-rank and ipc transports)
//   --restart PREFIX (start from fp64 checkpoint shards of any layout, Python or native:
//   diffusion runs `iters` more steps, Burgers continues to tEnd)  --checkpoint PREFIX
//   (write this run's shards at the end; checkpoint.cpp, the format of utils/io.py)
//   --style multigpu|singlegpu (summary block of the multi-GPU apps, default, or of the
//   single-GPU apps: no HtD/DtH lines, Final Time, SG GFLOPs convention)
//   --initial FILE (the starting field, float32 like result.bin: the reference's initial.bin)
//   --json (one metrics line with the keys of the Python front end's --json)
//   --warmup N (N untimed steps first, then the state as before them: Engine::warmup)
//   --config FILE.json (the keys of the Python front end's config files; see apply_config)
//   --ascii FILE (the result as one %g per line, fp64 values: the reference's Save3D, Tools.c:
//   66-86)  --print (the field as rows of %8.2f, a blank line between planes: Print3D)
//   --check-every N (NaN/Inf watchdog every N steps: a non-finite field stops every rank
//   with an error instead of running on; eager stepping)
//   --pitch PX,PY (pitched fields: PX extra elements per row, PY extra rows per 3-D plane;
//   default ADVDIFF_PITCH, else 4 fp64 / 16 fp32 elements + 1 row on 3-D fields past
//   128 MiB per rank)
// Launch one process per GPU with torchrun-style env vars (RANK/WORLD_SIZE/LOCAL_RANK/
// MASTER_ADDR/MASTER_PORT), e.g. via `python -m multigpu_advectiondiffusion_amd.launch`.
#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>

#include "runtime.hpp"

namespace advdiff::rt {

static int ic_code(const std::string& s) {
  static const std::map<std::string, int> m = {{"zero", 0},  {"square", 1},   {"sine", 2},
                                               {"heat", 3},  {"gaussian", 4}, {"plates", 5},
                                               {"disc", 6}};
  auto it = m.find(s);
  if (it == m.end()) throw std::runtime_error("unknown IC " + s);
  return it->second;
}

// --config FILE.json: a flat object, laid out like the Python front end's config files
// (cli.py _load_config): "args" = the positional list, every other key one of THESE
// options ("write-ghosts" or "write_ghosts"; true = a flag, false = absent).  Entries
// override the command line, as in cli.py.  TOML / YAML configs are the Python side's.
static void apply_config(const std::string& path, std::vector<std::string>& pos,
                         std::map<std::string, std::string>& opt) {
  if (path.size() < 5 || path.compare(path.size() - 5, 5, ".json") != 0)
    throw std::runtime_error("--config: the native apps read JSON configs (" + path + ")");
  std::ifstream f(path);
  if (!f) throw std::runtime_error("--config: cannot read " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string js = ss.str();
  size_t q = js.find('{');
  auto skip = [&] {
    while (q < js.size() && (std::isspace((unsigned char)js[q]) || js[q] == ',')) ++q;
  };
  auto string_at = [&]() {  // js[q] == '"'
    const size_t e = js.find('"', q + 1);
    if (e == std::string::npos) throw std::runtime_error("--config: bad JSON string");
    std::string v = js.substr(q + 1, e - q - 1);
    q = e + 1;
    return v;
  };
  auto scalar_at = [&]() {  // a string, number, true or false
    skip();
    if (q < js.size() && js[q] == '"') return string_at();
    const size_t b = q;
    while (q < js.size() && js[q] != ',' && js[q] != '}' && js[q] != ']' &&
           !std::isspace((unsigned char)js[q]))
      ++q;
    return js.substr(b, q - b);
  };
  if (q == std::string::npos) throw std::runtime_error("--config: not a JSON object");
  ++q;
  for (skip(); q < js.size() && js[q] != '}'; skip()) {
    if (js[q] != '"') throw std::runtime_error("--config: expected a key");
    std::string key = string_at();
    q = js.find(':', q);
    if (q == std::string::npos) throw std::runtime_error("--config: expected ':'");
    ++q;
    skip();
    if (key == "args") {
      if (js[q] != '[') throw std::runtime_error("--config: \"args\" must be a list");
      ++q;
      pos.clear();
      for (skip(); q < js.size() && js[q] != ']'; skip()) {
        const size_t q0 = q;
        pos.push_back(scalar_at());
        if (q == q0) throw std::runtime_error("--config: bad \"args\" list");
      }
      ++q;
      continue;
    }
    if (js[q] == '[' || js[q] == '{') throw std::runtime_error("--config: " + key + " must be a scalar");
    const size_t q0 = q;
    const std::string v = scalar_at();
    if (q == q0) throw std::runtime_error("--config: bad value of " + key);
    std::replace(key.begin(), key.end(), '_', '-');
    if (v == "false")
      opt.erase("--" + key);
    else
      opt["--" + key] = v == "true" ? "1" : v;
  }
}

int run_app(int argc, char** argv, Physics phys, int dims) {
  std::vector<std::string> pos;
  std::map<std::string, std::string> opt;
  for (int q = 1; q < argc; ++q) {
    std::string a = argv[q];
    if (a.rfind("--", 0) == 0) {
      const bool flag = a == "--fp32" || a == "--no-overlap" || a == "--boundary-on-comm" ||
                        a == "--no-boundary-on-comm" || a == "--fused-put" ||
                        a == "--error-norms" || a == "--no-fused" || a == "--geometry" || a == "--graph" ||
                        a == "--no-graph" || a == "--print" || a == "--json";
      if (flag || q + 1 >= argc) {
        opt[a] = "1";
      } else {
        opt[a] = argv[++q];
      }
    } else {
      pos.push_back(a);
    }
  }
  if (opt.count("--config")) apply_config(opt["--config"], pos, opt);
  const bool diff = phys == Physics::Diffusion;
  const size_t need = diff ? (dims == 3 ? 8 : 6) : (dims == 3 ? 8 : 6);
  if (pos.size() < need) {
    std::cerr << "usage: " << argv[0]
              << (diff ? (dims == 3 ? " K L W H Nx Ny Nz iters [bx by bz]" : " K L W Nx Ny iters [bx by]")
                       : (dims == 3 ? " tEnd CFL L W H Nx Ny Nz [bx by bz]" : " tEnd CFL L W Nx Ny [bx by]"))
              << " [--ic NAME] [--order 2|4] [--weno js|z|js7] [--integrator ssprk3|lsrk45] [--no-fused] [--visc C] [--fp32] [--no-overlap] [--[no-]boundary-on-comm] [--fused-put]"
                 " [--transport rccl|ipc|socket] [--decomp slab|PZxPYxPX|PYxPX] [--write FILE]"
                 " [--write-ghosts FILE] [--error-norms] [--geometry] [--graph|--no-graph]"
                 " [--restart PREFIX] [--checkpoint PREFIX] [--check-every N] [--ascii FILE]"
                 " [--print] [--config FILE.json] [--style multigpu|singlegpu] [--initial FILE]"
                 " [--json] [--warmup N] [--pitch PX,PY]\n";
    return 1;
  }
  Problem p;
  p.physics = phys;
  p.dims = dims;
  size_t k = 0;
  double tEnd = 0;
  int iters = 0;
  if (diff) {
    p.K = std::stod(pos[k++]);
  } else {
    tEnd = std::stod(pos[k++]);
    p.cfl = std::stod(pos[k++]);
  }
  p.L = std::stod(pos[k++]);
  p.W = std::stod(pos[k++]);
  if (dims == 3) p.H = std::stod(pos[k++]);
  p.nx = std::stoi(pos[k++]);
  p.ny = std::stoi(pos[k++]);
  if (dims == 3) p.nz = std::stoi(pos[k++]);
  if (diff) iters = std::stoi(pos[k++]);
  if (opt.count("--order")) p.order = std::stoi(opt["--order"]);
  if (opt.count("--safety")) p.safety = std::stod(opt["--safety"]);
  if (opt.count("--weno")) {
    const std::string w = opt["--weno"];
    if (w != "js" && w != "z" && w != "js7") throw std::runtime_error("--weno js|z|js7");
    p.weno = w == "js" ? 0 : (w == "z" ? 1 : 2);
  }
  if (opt.count("--integrator")) {
    const std::string g = opt["--integrator"];
    if (g != "ssprk3" && g != "lsrk45") throw std::runtime_error("--integrator ssprk3|lsrk45");
    p.integrator = g == "lsrk45" ? 1 : 0;
  }
  if (opt.count("--no-fused")) p.fused = false;
  if (opt.count("--visc")) p.C = std::stod(opt["--visc"]);
  if (opt.count("--fp32")) p.dtype = ADVDIFF_F32;
  if (opt.count("--no-overlap")) p.overlap = false;
  if (opt.count("--boundary-on-comm")) p.bcomm = 1;
  if (opt.count("--no-boundary-on-comm")) p.bcomm = 0;
  if (opt.count("--fused-put")) p.fused_put = 1;
  if (opt.count("--pitch")) {
    const std::string v = opt["--pitch"];
    if (std::sscanf(v.c_str(), "%d,%d", &p.pitch_px, &p.pitch_py) != 2 || p.pitch_px < 0 ||
        p.pitch_py < 0)
      throw std::runtime_error("--pitch PX,PY (extra elements per row, extra rows per plane)");
  }
  if (opt.count("--graph")) p.graph = 1;
  if (opt.count("--no-graph")) p.graph = 0;
  if (opt.count("--check-every")) p.check_every = std::stoi(opt["--check-every"]);
  const std::string decomp = opt.count("--decomp") ? opt["--decomp"] : "slab";
  std::string ic = opt.count("--ic") ? opt["--ic"] : (diff ? "heat" : "gaussian");
  p.ic = ic_code(ic);
  if (p.ic == 3) {
    p.ic_p0 = p.K;
    p.ic_p1 = 0.1;
    p.t0 = 0.1;
  } else if (p.ic == 4) {
    p.ic_p0 = 0.1;
  } else if (p.ic == 6) {
    p.ic_p0 = 0.2;
  }

  ProcEnv env = ProcEnv::from_env();
  if (opt.count("--geometry")) {  // host-only: the geometry every rank would use
    if (decomp != "slab") parse_pgrid(decomp, dims, env.size, p.pgrid);
    for (int r = 0; r < env.size; ++r) std::cout << geometry_json(p, r, env.size) << "\n";
    return 0;
  }
  int ndev = 0;
  HIP_CHECK(hipGetDeviceCount(&ndev));
  if (ndev == 0) throw std::runtime_error("no HIP device");
  const std::string tk = opt.count("--transport") ? opt["--transport"] : "rccl";
  if (env.size > ndev && tk != "socket" && tk != "ipc")
    throw std::runtime_error("more ranks than GPUs: one process per GPU (or --transport ipc|socket)");
  HIP_CHECK(hipSetDevice(env.local_rank % ndev));
  HIP_CHECK((hipError_t)advdiff_preload());  // code objects loaded before the timed loop
  if (decomp != "slab") parse_pgrid(decomp, dims, env.size, p.pgrid);
  auto tr = make_transport(env, tk);
  Engine eng(p, tr.get(), env);
  if (opt.count("--restart")) eng.load_checkpoint(opt["--restart"]);
  if (opt.count("--initial")) {  // the starting field (IC or restart), float32 like result.bin
    const std::vector<float> g0 = eng.gather_float32();
    if (env.rank == 0) write_binary(opt["--initial"], g0);
  }
  if (opt.count("--warmup")) eng.warmup(std::stoi(opt["--warmup"]));
  Stats st = diff ? eng.run_iters(iters) : eng.run_until(tEnd + p.t0);
  if (opt.count("--checkpoint")) eng.save_checkpoint(opt["--checkpoint"], ic);
  std::string title =
      std::string(diff ? "Diffusion-" : "Burgers-") + (dims == 3 ? "3D" : "2D") +
      (diff ? (p.order == 4 ? " MI355X-FD4" : " MI355X-FD2") : (p.weno == 1 ? " MI355X-WENO5Z" : p.weno == 0 ? " MI355X-WENO5JS" : " MI355X-WENO7JS"));
  std::string optname = std::string("Fused LDS z-march + RK3 (gfx950), transport=") + tr->name() +
                        (eng.graphs() ? ", hipGraph steps" : "") +
                        (eng.fused_puts() ? ", halo puts in the launch" : "");
  if (eng.cartesian()) {
    optname += ", decomp=" + std::to_string(eng.cart().pgrid[0]) + "x" +
               std::to_string(eng.cart().pgrid[1]);
    if (dims == 3) optname += "x" + std::to_string(eng.cart().pgrid[2]);
  }
  double l1 = 0, l2 = 0, li = 0;
  const bool norms = opt.count("--error-norms") && (p.ic == 2 || p.ic == 3);
  if (norms) eng.error_norms(l1, l2, li);
  // DtH: the barrier-fenced copy of the result to the host and — when an output needs the
  // global field (--write) — its gather to rank 0 (the reference's timed DtH +
  // Merge_domains, MultiGPU/Diffusion3d_Baseline/main.c:313-335).  Without one, each rank
  // times the copy of its own block only: no full-field copy on rank 0's host, no merge
  // over the TCP star (at 2048^3 that would be ~70 GB per run for nothing)
  auto wall = [] {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  tr->barrier();
  const double tw = wall();
  std::vector<float> g;
  if (opt.count("--write"))
    g = eng.gather_float32();
  else
    eng.dtoh_local();
  tr->barrier();
  st.dtoh = tr->allreduce_max(wall() - tw);
  std::vector<float> gg;
  if (opt.count("--write-ghosts")) gg = eng.gather_float32_ghosts();
  std::vector<double> gd;  // fp64 text output, formatted as utils/io.py does
  if (opt.count("--ascii") || opt.count("--print")) gd = eng.gather_float64();
  if (env.rank == 0) {
    std::cout << "advdiff native build: runtime " << advdiff_runtime_hash() << ", kernels "
              << advdiff_source_hash() << "\n";
    if (pos.size() > need) std::cout << "(block sizes ignored: gfx950 tiles are fixed)\n";
    const std::string style = opt.count("--style") ? opt["--style"] : "multigpu";
    if (style == "singlegpu") {  // the single-GPU apps' block, norms inside it (cli.py)
      auto f = [](const char* spec, double v) {
        char b[64];
        std::snprintf(b, sizeof b, spec, v);
        return std::string(b);
      };
      const double ml = st.seconds > 0 ? p.cells() * (double)st.steps / st.seconds / 1e6 : 0;
      std::vector<std::pair<std::string, std::string>> ex = {
          {"MLUPS (cells x RK3 steps / s)", f("%.1f", ml)},
          {"Stage-MLUPS", f("%.1f", 3 * ml)},
          {"Processes / devices", std::to_string(env.size) + " x gfx950"}};
      if (norms) {
        ex.push_back({"L1 norm", f("%e", l1)});
        ex.push_back({"L2 norm", f("%e", l2)});
        ex.push_back({"Linf norm", f("%e", li)});
      }
      std::cout << summary_singlegpu(title, optname, st, p, ex);
    } else {
      std::cout << summary_multigpu(title, optname, st, p, env.size);
      if (norms) {
        std::printf("L1 norm                                       :  %e\n", l1);
        std::printf("L2 norm                                       :  %e\n", l2);
        std::printf("Linf norm                                     :  %e\n", li);
      }
    }
    if (opt.count("--write")) write_binary(opt["--write"], g);
    if (opt.count("--write-ghosts")) write_binary(opt["--write-ghosts"], gg);
    if (opt.count("--ascii")) {
      FILE* f = std::fopen(opt["--ascii"].c_str(), "w");
      if (f == nullptr) throw std::runtime_error("cannot write " + opt["--ascii"]);
      for (double v : gd) std::fprintf(f, "%g\n", v);
      std::fclose(f);
    }
    if (opt.count("--print")) {
      const int nx = p.nx, ny = p.ny;  // 3-D: nz planes of ny rows; 2-D: one plane
      const size_t plane = (size_t)nx * ny;
      std::string txt;
      char cell[64];
      for (size_t k = 0; k * plane < gd.size(); ++k) {
        for (int j = 0; j < ny; ++j) {
          for (int i = 0; i < nx; ++i) {
            std::snprintf(cell, sizeof cell, "%8.2f", gd[k * plane + (size_t)j * nx + i]);
            txt += cell;
          }
          txt += "\n";
        }
        txt += "\n";
      }
      std::cout << txt << "\n";
    }
    if (opt.count("--json")) {  // one metrics line, the keys of cli.py --json
      const double ml = st.seconds > 0 ? p.cells() * (double)st.steps / st.seconds / 1e6 : 0;
      char line[512];
      const std::string grid = "[" + std::to_string(p.nx) + ", " + std::to_string(p.ny) +
                               (dims == 3 ? ", " + std::to_string(p.nz) : std::string()) + "]";
      std::snprintf(line, sizeof line,
                    "{\"app\": \"%s\", \"grid\": %s, \"steps\": %d, \"seconds\": %.17g, "
                    "\"mlups\": %.17g, \"n_procs\": %d, \"dtype\": \"%s\", \"t\": %.17g, "
                    "\"device_field_bytes\": %zu}",
                    (std::string(diff ? "diffusion" : "burgers") + (dims == 3 ? "3d" : "2d")).c_str(),
                    grid.c_str(), st.steps, st.seconds, ml, env.size,
                    p.dtype == ADVDIFF_F64 ? "fp64" : "fp32", st.t, eng.memory_bytes());
      std::cout << line << "\n";
    }
    std::cout.flush();
  }
  tr->barrier();
  return 0;
}

}  // namespace advdiff::rt
