// uncomp -- drop-in for AntiZ's CLI (main.cpp:1066-1231) on top of libatz_accel (MI355X).
// Same switches (parseCLI, main.cpp:1070-1143), same default file names (.atz / .rec), same stdout
// lines and exit codes; the work goes through the C ABI in include/atz_accel.h.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "atz_accel.h"

#define ANTIZ_VER "0.1.6-git"

static bool read_file(const std::string& n, std::vector<uint8_t>& v) {
  std::ifstream f(n, std::ios::binary);
  if (!f.is_open()) return false;
  f.seekg(0, f.end);
  std::streamoff sz = f.tellg();
  f.seekg(0, f.beg);
  v.resize((size_t)sz);
  if (sz) f.read(reinterpret_cast<char*>(v.data()), sz);
  return true;
}
static bool write_file(const std::string& n, const uint8_t* p, uint64_t len) {
  std::ofstream f(n, std::ios::binary | std::ios::trunc);
  if (!f.is_open()) return false;
  f.write(reinterpret_cast<const char*>(p), (std::streamsize)len);
  return (bool)f;
}

static void usage(const char* argv0) {
  std::cout << "\nUSAGE: \n\n   " << argv0
            << "  [--brute-window] [--notest] [-r] [--chunksize <integer>] [--mismatch-tol <integer>]"
               " [--shortcut-len <integer>] [--sizediff-tresh <integer>] [--recomp-tresh <integer>]"
               " [-o <string>] -i <string> [--] [--version] [-h]\n";
}

int main(int argc, char* argv[]) {
  std::cout << "AntiZ " << ANTIZ_VER << std::endl;
  atz_opts_t o;
  atz_default_opts(&o);
  std::string in, out;
  bool recon = false, notest = false, have_out = false, have_in = false;
  for (int k = 1; k < argc; k++) {
    std::string a = argv[k];
    auto val = [&](const char* name) -> std::string {
      if (k + 1 >= argc) {
        std::cerr << "PARSE ERROR: Argument: " << name << "\n             Missing a value for this argument!\n";
        usage(argv[0]);
        std::exit(1);
      }
      return argv[++k];
    };
    if (a == "-i" || a == "--input") { in = val("-i"); have_in = true; }
    else if (a == "-o" || a == "--output") { out = val("-o"); have_out = true; }
    else if (a == "-r" || a == "--reconstruct") recon = true;
    else if (a == "--notest") notest = true;
    else if (a == "--brute-window") o.brute_window = 1;
    else if (a == "--recomp-tresh") o.recomp_tresh = std::strtoull(val("--recomp-tresh").c_str(), nullptr, 10);
    else if (a == "--sizediff-tresh") o.sizediff_tresh = std::strtoull(val("--sizediff-tresh").c_str(), nullptr, 10);
    else if (a == "--shortcut-len") o.shortcut_len = std::strtoull(val("--shortcut-len").c_str(), nullptr, 10);
    else if (a == "--mismatch-tol") o.mismatch_tol = std::strtoull(val("--mismatch-tol").c_str(), nullptr, 10);
    else if (a == "--chunksize") o.chunksize = std::strtoull(val("--chunksize").c_str(), nullptr, 10);
    else if (a == "--device") o.device = std::atoi(val("--device").c_str());
    else if (a == "--version") { std::cout << "\n" << argv[0] << "  version: " << ANTIZ_VER << "\n\n"; return 0; }
    else if (a == "-h" || a == "--help") { usage(argv[0]); return 0; }
    else if (a == "--") continue;
    else {
      std::cerr << "PARSE ERROR: Argument: " << a << "\n             Couldn't find match for argument\n";
      usage(argv[0]);
      return 1;
    }
  }
  if (!have_in) {
    std::cerr << "PARSE ERROR:  \n             Required argument missing: input\n";
    usage(argv[0]);
    return 1;
  }
  std::cout << "Input file: " << in << std::endl;
  std::string atzname, recname;
  if (recon) {
    std::cout << "assuming input file is an ATZ file, attempting to reconstruct" << std::endl;
    atzname = in;
    recname = have_out ? out : in + ".rec";
    std::cout << "overwriting " << recname << " if present" << std::endl;
  } else {
    atzname = have_out ? out : in + ".atz";
    recname = in + ".rec";
    std::cout << "overwriting " << atzname << " and " << recname << " if present" << std::endl;
  }
  atz_ctx_t* ctx = nullptr;
  int rc = atz_open(&ctx, &o);
  if (rc) { std::cerr << "atz: " << atz_strerror(rc) << std::endl; return 255; }
  auto reconstruct = [&](const std::string& a, const std::string& r) -> int {
    std::cout << "reconstructing from " << a << std::endl;
    std::vector<uint8_t> az;
    if (!read_file(a, az)) { std::cout << "error: open file for size check failed!" << std::endl; return -1; }
    if (az.size() < 4 || std::memcmp(az.data(), "ATZ\1", 4) != 0) {
      std::cout << "Invalid file: ATZ1 header not found" << std::endl;
      return -2;
    }
    uint64_t flen = 0;
    if (az.size() >= 12) std::memcpy(&flen, az.data() + 4, 8);
    if (flen != az.size()) { std::cout << "Invalid file: ATZ file size mismatch" << std::endl; return -3; }
    uint64_t orig = 0;
    if (az.size() >= 20) std::memcpy(&orig, az.data() + 12, 8);
    std::cout << "ATZ file size: " << az.size() << std::endl;
    std::cout << "Original file size: " << orig << std::endl;
    uint8_t* rec = nullptr;
    uint64_t rl = 0;
    int e = atz_reconstruct(ctx, az.data(), az.size(), &rec, &rl);
    if (e) { std::cerr << "atz: " << atz_strerror(e) << std::endl; return -1; }
    bool ok = write_file(r, rec, rl);
    atz_free(rec);
    return ok ? 0 : -1;
  };
  int ret = 0;
  if (!recon) {
    std::vector<uint8_t> data;
    if (!read_file(in, data)) {
      std::cerr << "Error Encountered: " << "failed to open File " << in << std::endl;
      atz_close(ctx);
      return 1;
    }
    uint8_t* atz = nullptr;
    uint64_t al = 0;
    atz_stats_t st;
    rc = atz_precompress(ctx, data.data(), data.size(), &atz, &al, &st);
    if (rc) {
      std::cerr << "atz: " << atz_strerror(rc) << std::endl;
      atz_close(ctx);
      return rc == ATZ_E_REF_ABORT ? 134 : 255;
    }
    std::cout << "Total zlib headers found: " << st.n_streams << std::endl;
    std::cout << std::endl;
    std::cout << "recompressed:" << st.n_recomp << "/" << st.n_streams << std::endl;
    if (!write_file(atzname, atz, al)) { std::cout << "error: open file for output failed!" << std::endl; return 134; }
    std::cout << "Total bytes written: " << al << std::endl;
    atz_free(atz);
    if (!notest) {
      if (reconstruct(atzname, recname) != 0) {
        std::cerr << "Error Encountered: " << "testATZFile() : Reconstruction Failed" << std::endl;
        atz_close(ctx);
        return 1;
      }
      std::cout << "Testing...";
      std::vector<uint8_t> rec;
      read_file(recname, rec);
      if (rec.size() != data.size()) { std::cout << "error: size mismatch"; ret = -1; }
      else if (rec != data) { std::cout << "error: byte mismatch"; ret = -1; }
      else {
        std::cout << "OK! Restoration is bit by bit identical" << std::endl;
        if (std::remove(recname.c_str()) != 0) { std::cout << "error: cannot delete recfile"; ret = -1; }
      }
    }
  } else {
    if (reconstruct(atzname, recname) != 0) ret = -1;
  }
  atz_close(ctx);
  return ret;
}
