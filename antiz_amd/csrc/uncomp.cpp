// uncomp -- drop-in for AntiZ's CLI (main.cpp:1066-1231) on top of libatz_accel (MI355X).
// Same switches (parseCLI, main.cpp:1070-1143), same default file names (.atz / .rec), same stdout
// and stderr lines and exit codes; the work goes through the C ABI in include/atz_accel.h.
//
// The reference parses with TCLAP 1.2.1 (vendored, header-only).  Its observable behaviour for this
// one fixed argument set is restated below (the parse loop, the switch/value matching rules, the
// error texts and the help/usage layout), so every CLI path -- -h, --version, parse errors, bad
// integers, "--" -- prints what the reference prints:
//   T/ = includes, tools, stuff/tclap/tclap-1.2.1/include/tclap/
//   CmdLine::parse            T/CmdLine.h:444-509   (loop, _emptyCombined 511-521, missing args 523-548)
//   ValueArg::processArg      T/ValueArg.h:327-370  (trimFlag T/Arg.h:620-636, _hasBlanks 641-648)
//   SwitchArg::processArg     T/SwitchArg.h:228-257 (combined switches 164-204, lastCombined 155-162)
//   ExtractValue (ValueLike)  T/Arg.h:414-443       (istream >> value; trailing junk / 2 values fail)
//   StdOutput                 T/StdOutput.h:108-295 (version, usage, failure, spacePrint)
// The context is opened only when GPU work starts, so every parse and file error path runs without
// a GPU (tests/test_cli.py checks them against the reference's own output).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "atz_accel.h"

#define ANTIZ_VER "0.1.6-git"

namespace cli {

// One argument of the reference's command line (main.cpp:1078-1102 plus TCLAP's own three).
struct Arg {
  enum Kind { SWITCH, STRING, UINT };
  enum Role { PLAIN, HELP, VERSION, IGNORE_REST };
  std::string flag;   // one character or empty
  std::string name;
  std::string desc;
  Kind kind;
  bool required;
  Role role;
  bool set = false;
  std::string sval;
  uint64_t uval = 0;

  std::string flag_id() const { return "-" + flag; }
  std::string name_id() const { return "--" + name; }
  bool takes_value() const { return kind != SWITCH; }
  std::string type_desc() const { return kind == STRING ? "string" : "integer"; }
  bool matches(const std::string& s) const {
    return (!flag.empty() && s == flag_id()) || s == name_id();
  }
  std::string to_string() const { return (flag.empty() ? "" : flag_id() + " ") + "(" + name_id() + ")"; }
  std::string short_id() const {
    std::string id = flag.empty() ? name_id() : flag_id();
    if (takes_value()) id += " <" + type_desc() + ">";
    return required ? id : "[" + id + "]";
  }
  std::string long_id() const {
    std::string id;
    if (!flag.empty()) {
      id = flag_id();
      if (takes_value()) id += " <" + type_desc() + ">";
      id += ",  ";
    }
    id += name_id();
    if (takes_value()) id += " <" + type_desc() + ">";
    return id;
  }
  std::string description() const { return required ? "(required)  " + desc : desc; }
};

struct ParseError {
  std::string id;   // empty: no argument named ("PARSE ERROR:  ")
  std::string text;
};
struct Exit {
  int status;
};

const char kBlank = 7;   // marks a consumed letter of a combined switch (TCLAP's blankChar)

struct CmdLine {
  std::vector<Arg> args;   // in TCLAP's list order: the last one added comes first
  std::string prog;
  std::string message = "Visit https://github.com/Diazonium/AntiZ for source code and support.";
  bool ignoring = false;

  Arg& get(const char* name) {
    for (auto& a : args)
      if (a.name == name) return a;
    std::abort();
  }

  // Line-wraps s at spaces, commas and pipes (StdOutput::spacePrint).
  static void space_print(std::ostream& os, const std::string& s, int max_width, int indent, int second_off) {
    const int len = (int)s.size();
    auto at = [&](int k) { return k < len ? s[k] : '\0'; };
    if (len + indent <= max_width) {
      os << std::string(indent, ' ') << s << std::endl;
      return;
    }
    int allowed = max_width - indent;
    int start = 0;
    while (start < len) {
      int n = std::min(len - start, allowed);
      if (n == allowed)
        while (n >= 0 && at(n + start) != ' ' && at(n + start) != ',' && at(n + start) != '|') n--;
      if (n <= 0) n = allowed;
      for (int k = 0; k < n; k++)
        if (s[start + k] == '\n') n = k + 1;
      os << std::string(indent, ' ');
      if (start == 0) {
        indent += second_off;
        allowed -= second_off;
      }
      os << s.substr(start, n) << std::endl;
      while (at(n + start) == ' ' && start < len) start++;
      start += n;
    }
  }
  void short_usage(std::ostream& os) const {
    std::string s = prog + " ";
    for (const auto& a : args) s += " " + a.short_id();
    int off = std::min((int)prog.size() + 2, 75 / 2);
    space_print(os, s, 75, 3, off);
  }
  void long_usage(std::ostream& os) const {
    for (const auto& a : args) {
      space_print(os, a.long_id(), 75, 3, 3);
      space_print(os, a.description(), 75, 5, 0);
      os << std::endl;
    }
    os << std::endl;
    space_print(os, message, 75, 3, 0);
  }
  void usage() const {
    std::cout << std::endl << "USAGE: " << std::endl << std::endl;
    short_usage(std::cout);
    std::cout << std::endl << std::endl << "Where: " << std::endl << std::endl;
    long_usage(std::cout);
    std::cout << std::endl;
  }
  void version() const { std::cout << std::endl << prog << "  version: " << ANTIZ_VER << std::endl << std::endl; }
  void failure(const ParseError& e) const {
    std::cerr << "PARSE ERROR: " << (e.id.empty() ? std::string(" ") : "Argument: " + e.id) << std::endl
              << "             " << e.text << std::endl << std::endl;
    std::cerr << "Brief USAGE: " << std::endl;
    short_usage(std::cerr);
    std::cerr << std::endl << "For complete USAGE and HELP type: " << std::endl
              << "   " << prog << " --help" << std::endl << std::endl;
  }

  // A switch took effect: set it once, then run its action (help/version exit, "--" ignores the rest).
  void fire(Arg& a) {
    if (a.set) throw ParseError{a.to_string(), "Argument already set!"};
    a.set = true;
    if (a.role == Arg::HELP) { usage(); throw Exit{0}; }
    if (a.role == Arg::VERSION) { version(); throw Exit{0}; }
    if (a.role == Arg::IGNORE_REST) ignoring = true;
  }

  // One letter of a combined switch like "-rh" (consumed letters are blanked in place).
  static bool combined_take(const Arg& a, std::string& s) {
    if (!s.empty() && s[0] != '-') return false;
    if (s.compare(0, 2, "--") == 0) return false;
    if (s.find(' ') != std::string::npos) return false;
    for (size_t k = 1; k < s.size(); k++)
      if (!a.flag.empty() && s[k] == a.flag[0] && a.flag[0] != '-') {
        s[k] = kBlank;
        return true;
      }
    return false;
  }
  static bool only_blanks_after_first(const std::string& s) {
    for (size_t k = 1; k < s.size(); k++)
      if (s[k] != kBlank) return false;
    return true;
  }

  static void extract(Arg& a, const std::string& v) {
    if (a.kind == Arg::STRING) {
      a.sval = v;
      return;
    }
    std::istringstream is(v);
    unsigned long x = a.uval;   // an empty string leaves the default
    int n_read = 0;
    while (is.good()) {
      if (is.peek() == EOF) break;
      is >> x;
      n_read++;
    }
    if (is.fail()) throw ParseError{a.to_string(), "Couldn't read argument value from string '" + v + "'"};
    if (n_read > 1) throw ParseError{a.to_string(), "More than one valid value parsed from string '" + v + "'"};
    a.uval = x;
  }

  // Returns whether args[i] was taken by a (i advances past a value).
  bool take(Arg& a, std::vector<std::string>& av, size_t& i) {
    if (ignoring) return false;
    if (a.kind == Arg::SWITCH) {
      if (a.matches(av[i])) {
        fire(a);
        return true;
      }
      if (combined_take(a, av[i])) {
        if (combined_take(a, av[i])) throw ParseError{a.to_string(), "Argument already set!"};
        fire(a);
        return only_blanks_after_first(av[i]);
      }
      return false;
    }
    for (size_t k = 1; k < av[i].size(); k++)
      if (av[i][k] == kBlank) return false;
    std::string flag = av[i], value;
    size_t sp = flag.find(' ');
    if (sp != std::string::npos && sp > 1) {
      value = flag.substr(sp + 1);
      flag = flag.substr(0, sp);
    }
    if (!a.matches(flag)) return false;
    if (a.set) throw ParseError{a.to_string(), "Argument already set!"};
    if (value.empty()) {
      if (++i >= av.size()) throw ParseError{a.to_string(), "Missing a value for this argument!"};
      extract(a, av[i]);
    } else {
      extract(a, value);
    }
    a.set = true;
    return true;
  }

  void parse(int argc, char** argv) {
    std::vector<std::string> av(argv, argv + argc);
    prog = av.front();
    av.erase(av.begin());
    int n_required = 0, seen_required = 0;
    for (const auto& a : args) n_required += a.required;
    for (size_t i = 0; i < av.size(); i++) {
      bool matched = false;
      for (auto& a : args)
        if (take(a, av, i)) {
          seen_required += a.required;
          matched = true;
          break;
        }
      if (!matched && (av[i].empty() || av[i][0] == '-') && only_blanks_after_first(av[i])) matched = true;
      if (!matched && !ignoring) throw ParseError{av[i], "Couldn't find match for argument"};
    }
    if (seen_required < n_required) {
      std::string missing;
      int n = 0;
      for (const auto& a : args)
        if (a.required && !a.set) {
          missing += (n++ ? ", " : "") + a.name;
        }
      throw ParseError{"", (n > 1 ? "Required arguments missing: " : "Required argument missing: ") + missing};
    }
  }
};

CmdLine make_cmdline() {
  CmdLine c;
  auto add = [&](const char* f, const char* n, Arg::Kind k, bool req, const char* d, Arg::Role r = Arg::PLAIN) {
    Arg a;
    a.flag = f;
    a.name = n;
    a.kind = k;
    a.required = req;
    a.desc = d;
    a.role = r;
    c.args.insert(c.args.begin(), a);
  };
  add("h", "help", Arg::SWITCH, false, "Displays usage information and exits.", Arg::HELP);
  add("", "version", Arg::SWITCH, false, "Displays version information and exits.", Arg::VERSION);
  add("-", "ignore_rest", Arg::SWITCH, false, "Ignores the rest of the labeled arguments following this flag.",
      Arg::IGNORE_REST);
  add("i", "input", Arg::STRING, true, "Input file name");
  add("o", "output", Arg::STRING, false, "Output file name");
  add("", "recomp-tresh", Arg::UINT, false,
      "Recompression treshold in bytes. Streams are only recompressed if the best match differs from the "
      "original in at most recompTresh bytes. Increasing this treshold may allow more streams to be "
      "recompressed, but may increase ATZ file overhead and make it harder to compress. Default: 128  "
      "Maximum: 65535");
  add("", "sizediff-tresh", Arg::UINT, false,
      "Size difference treshold in bytes. If the size difference between a recompressed stream and the "
      "original is more than the treshold then do not even compare them. Increasing this treshold increases "
      "the chance that a stream will be compared to the original. The cost of comparing is relatively low, so "
      "setting this equal to the recompression treshold should be fine. Default: 128  Maximum: 65535");
  add("", "shortcut-len", Arg::UINT, false,
      "Length of the shortcut in bytes. If a stream is longer than the shortcut, then stop compression after "
      "<shortcut> compressed bytes have been obtained and compare this portion to the original. If this "
      "comparison yields more than recompTresh mismatches, then do not compress the entire stream. Lowering "
      "this improves speed, but it must be significantly greater than recompTresh or the speed benefit will "
      "decrease. Default: 512  Maximum: 65535");
  add("", "mismatch-tol", Arg::UINT, false,
      "Mismatch tolerance in bytes. If a set of parameters are found that give at most this many "
      "mismatches, then accept them and stop looking for a better set of parameters. Increasing this "
      "improves speed at the cost of more ATZ file overhead that may hurt compression. Default: 2  "
      "Maximum: 65535");
  add("", "chunksize", Arg::UINT, false,
      "Size of the memory buffer in bytes for chunked disk IO. This contorls memory usage to some extent, "
      "but memory usage control is not fully implemented yet. Smaller values result in more disk IO "
      "operations. Default: 524288");
  add("r", "reconstruct", Arg::SWITCH, false,
      "Assume the input file is an ATZ file and attempt to reconstruct the original file from it");
  add("", "notest", Arg::SWITCH, false,
      "Skip comparing the reconstructed file to the original at the end. This is not recommended, as AntiZ "
      "is still experimental software and my contain bugs that corrupt data.");
  add("", "brute-window", Arg::SWITCH, false,
      "Bruteforce deflate window size if there is a chance that recompression could be improved by it. This "
      "can have a major performance penalty. Default: disabled");
  c.get("recomp-tresh").uval = 128;
  c.get("sizediff-tresh").uval = 128;
  c.get("shortcut-len").uval = 512;
  c.get("mismatch-tol").uval = 2;
  c.get("chunksize").uval = 524288;
  return c;
}

}  // namespace cli

static bool read_file(const std::string& n, std::vector<uint8_t>& v) {
  std::ifstream f(n, std::ios::binary);
  if (!f.is_open()) return false;
  f.seekg(0, f.end);
  std::streamoff sz = f.tellg();
  f.seekg(0, f.beg);
  if (sz < 0) return false;
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

int main(int argc, char* argv[]) {
  std::cout << "AntiZ " << ANTIZ_VER << std::endl;
  cli::CmdLine cmd = cli::make_cmdline();
  try {
    cmd.parse(argc, argv);
  } catch (const cli::ParseError& e) {
    cmd.failure(e);
    std::exit(1);
  } catch (const cli::Exit& e) {
    std::exit(e.status);
  }
  atz_opts_t o;
  atz_default_opts(&o);
  o.recomp_tresh = cmd.get("recomp-tresh").uval;
  o.sizediff_tresh = cmd.get("sizediff-tresh").uval;
  o.shortcut_len = cmd.get("shortcut-len").uval;
  o.mismatch_tol = cmd.get("mismatch-tol").uval;
  o.chunksize = cmd.get("chunksize").uval;
  o.brute_window = cmd.get("brute-window").set ? 1 : 0;
  if (const char* dev = std::getenv("ATZ_DEVICE")) o.device = std::atoi(dev);   // not a reference flag
  const std::string in = cmd.get("input").sval;
  const bool have_out = cmd.get("output").set, recon = cmd.get("reconstruct").set, notest = cmd.get("notest").set;
  const std::string out = cmd.get("output").sval;

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
  auto open_ctx = [&]() -> int {
    if (ctx) return 0;
    int rc = atz_open(&ctx, &o);
    if (rc) std::cerr << "atz: " << atz_strerror(rc) << std::endl;
    return rc;
  };
  auto done = [&](int rc) {
    if (ctx) atz_close(ctx);
    return rc;
  };
  // ATZreconstructor::reconstructATZ (main.cpp:869-950) with parseATZheader's checks (1011-1030).
  auto reconstruct = [&](const std::string& a, const std::string& r) -> int {
    std::cout << "reconstructing from " << a << std::endl;
    std::vector<uint8_t> az;
    if (!read_file(a, az)) {
      std::cout << "error: open file for size check failed!" << std::endl;
      std::cout << "Cannot open file: " << a << std::endl;
      return -1;
    }
    if (az.size() < 4 || std::memcmp(az.data(), "ATZ\1", 4) != 0) {
      std::cout << "Invalid file: ATZ1 header not found" << std::endl;
      return -2;
    }
    uint64_t flen = 0;
    if (az.size() >= 12) std::memcpy(&flen, az.data() + 4, 8);
    if (flen != az.size()) {
      std::cout << "Invalid file: ATZ file size mismatch" << std::endl;
      return -3;
    }
    uint64_t orig = 0;
    if (az.size() >= 20) std::memcpy(&orig, az.data() + 12, 8);
    std::cout << "ATZ file size: " << az.size() << std::endl;
    std::cout << "Original file size: " << orig << std::endl;
    if (open_ctx()) return -1;
    uint8_t* rec = nullptr;
    uint64_t rl = 0;
    int e = atz_reconstruct(ctx, az.data(), az.size(), &rec, &rl);
    if (e) {
      std::cerr << "atz: " << atz_strerror(e) << std::endl;
      return -1;
    }
    bool ok = write_file(r, rec, rl);
    atz_free(rec);
    return ok ? 0 : -1;
  };

  if (recon) return done(reconstruct(atzname, recname) != 0 ? 255 : 0);

  // searchInfile's open check (main.cpp:401-402) comes before any output of Phase 1.
  std::vector<uint8_t> data;
  if (!read_file(in, data)) {
    std::cerr << "Error Encountered: " << "failed to open File " << in << std::endl;
    return done(1);
  }
  if (open_ctx()) return done(255);
  uint8_t* atz = nullptr;
  uint64_t al = 0;
  atz_stats_t st;
  int rc = atz_precompress(ctx, data.data(), data.size(), &atz, &al, &st);
  if (rc) {
    std::cerr << "atz: " << atz_strerror(rc) << std::endl;
    return done(rc == ATZ_E_REF_ABORT ? 134 : 255);
  }
  std::cout << "Total zlib headers found: " << st.n_streams << std::endl;
  std::cout << std::endl;
  std::cout << "recompressed:" << st.n_recomp << "/" << st.n_streams << std::endl;
  if (!write_file(atzname, atz, al)) {
    std::cout << "error: open file for output failed!" << std::endl;
    atz_free(atz);
    return done(134);
  }
  std::cout << "Total bytes written: " << al << std::endl;
  atz_free(atz);
  if (notest) return done(0);
  // testATZfile (main.cpp:1173-1203)
  if (reconstruct(atzname, recname) != 0) {
    std::cerr << "Error Encountered: " << "testATZFile() : Reconstruction Failed" << std::endl;
    return done(1);
  }
  std::cout << "Testing...";
  std::vector<uint8_t> rec;
  read_file(recname, rec);
  if (rec.size() != data.size()) {
    std::cout << "error: size mismatch";
    return done(255);
  }
  if (rec != data) {
    std::cout << "error: byte mismatch";
    return done(255);
  }
  std::cout << "OK! Restoration is bit by bit identical" << std::endl;
  if (std::remove(recname.c_str()) != 0) {
    std::cout << "error: cannot delete recfile";
    return done(255);
  }
  return done(0);
}
