// C++ host above the C ABI, shaped like the reference's in-process bench loop
// (engine_bench.cc:255-279): load an index, run the queries of a log file
// (query_pool.h:319-378 format: one query per line, terms separated by spaces)
// and print "doc:score(hex)" per hit.  Used by tests/test_cpp_host.py.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>

#include "wiser_hip_engine.hpp"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "usage: engine_cli <index dir> <query log> [k] [snippets]\n";
    return 2;
  }
  const int k = argc > 3 ? std::atoi(argv[3]) : 10;
  // "snippets": SearchQuery::return_snippets; each result line is followed by
  // one line of the entries' snippets, hex encoded, comma separated
  const bool snippets = argc > 4 && std::string(argv[4]) == "snippets";
  try {
    wiser_hip::VacuumHipEngine eng(argv[1]);
    eng.Load();
    std::vector<wiser_hip::SearchQuery> qs;
    std::ifstream in(argv[2]);
    for (std::string line; std::getline(in, line);) {
      std::istringstream ss(line);
      wiser_hip::SearchQuery q;
      for (std::string t; ss >> t;) q.terms.push_back(t);
      q.n_results = k;
      q.return_snippets = snippets;
      qs.push_back(q);
    }
    auto res = eng.SearchBatch(qs);
    for (auto& r : res) {
      for (size_t i = 0; i < r.Size(); ++i)
        std::printf("%s%d:%a", i ? " " : "", r[i].doc_id, r[i].doc_score);
      std::printf("\n");
      if (snippets) {
        for (size_t i = 0; i < r.Size(); ++i) {
          std::printf("%s", i ? "," : "");
          for (unsigned char c : r[i].snippet) std::printf("%02x", c);
        }
        std::printf("\n");
      }
    }
    std::cerr << "terms " << eng.TermCount() << "\n";
  } catch (const std::exception& e) {
    std::cerr << e.what() << "\n";
    return 1;
  }
  return 0;
}
