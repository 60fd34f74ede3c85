// CPU check of the engine's term dictionary (wiser_amd/csrc/index.cc): reads
// terms from stdin, one per line, and prints for each
//   <term> <id by find()> <id by find_many()> <df or 0>
// so tests/test_dictionary.py can compare both lookup paths with the oracle's
// own reading of my.tip.  Also checks that every term of the dictionary finds
// its own id.  Usage: dict_check <vacuum_dir>
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

#include "../../wiser_amd/csrc/index.h"

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s <vacuum_dir>\n", argv[0]);
    return 2;
  }
  wiser::VacuumIndex idx;
  idx.open(argv[1]);
  for (int32_t id = 0; id < idx.n_lists(); ++id)
    if (idx.find(idx.term(id)) != id) {
      std::fprintf(stderr, "term %d '%s' finds %d\n", id, idx.term(id).c_str(), idx.find(idx.term(id)));
      return 1;
    }
  std::vector<std::string> terms;
  for (std::string line; std::getline(std::cin, line);) terms.push_back(line);
  std::vector<const char*> p;
  std::vector<uint32_t> n;
  for (const auto& t : terms) {
    p.push_back(t.data());
    n.push_back(static_cast<uint32_t>(t.size()));
  }
  std::vector<int32_t> many(terms.size());
  idx.find_many(p.data(), n.data(), terms.size(), many.data());
  for (size_t i = 0; i < terms.size(); ++i) {
    const int32_t one = idx.find(terms[i]);
    std::printf("%s %d %d %u\n", terms[i].c_str(), one, many[i], one >= 0 ? idx.df(one) : 0u);
  }
  std::fprintf(stderr, "dict_check: %d lists, %zu queries\n", idx.n_lists(), terms.size());
  return 0;
}
