// Weighted edge-list loader: the graph file the
// reference's builder writes with nx.write_weighted_edgelist
// (build_graph.py:199) -> the symmetric adjacency trainer.py builds from it
// (nx.read_weighted_edgelist(nodetype=int) :98, adjacency_matrix(nodelist =
// range(n), dtype float32) :102-112, max(A, A^T) :148), as an int32 CSR with
// sorted, duplicate-free columns -- no networkx on the load path.
//
// Format: one edge per line, "u v w" (integer node ids, decimal weight),
// blank lines and '#' comments skipped.  The graph is undirected: A[u][v] =
// A[v][u] = float32(w) (parsed as double like Python's float(), rounded once);
// a repeated edge keeps the last weight (networkx add_edge overwrites).
// Node ids must be 0..n-1 with n = the number of distinct ids (what
// nodelist = range(number_of_nodes) requires).
#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <vector>

#include "gcnk_common.h"

namespace gcnk {
namespace {

struct Edge {
  int64_t u, v;
  int64_t order;
  float w;
};

int parse(const char* path, std::vector<Edge>& edges, int64_t& n) {
  FILE* f = std::fopen(path, "r");
  if (!f) {
    set_error("gcnk_edgelist: cannot open %s: %s", path, std::strerror(errno));
    return GCNK_EARG;
  }
  std::vector<char> line(1 << 16);
  int64_t lineno = 0, maxid = -1;
  edges.clear();
  while (std::fgets(line.data(), (int)line.size(), f)) {
    ++lineno;
    char* p = line.data();
    while (*p == ' ' || *p == '\t') ++p;
    if (*p == '\0' || *p == '\n' || *p == '\r' || *p == '#') continue;
    char* end = nullptr;
    const long long u = std::strtoll(p, &end, 10);
    if (end == p) goto bad;
    p = end;
    {
      const long long v = std::strtoll(p, &end, 10);
      if (end == p) goto bad;
      p = end;
      const double w = std::strtod(p, &end);
      if (end == p || u < 0 || v < 0) goto bad;
      edges.push_back({u, v, (int64_t)edges.size(), (float)w});
      maxid = std::max<int64_t>(maxid, std::max<int64_t>(u, v));
      continue;
    }
  bad:
    std::fclose(f);
    set_error("gcnk_edgelist: %s:%lld: expected \"u v weight\"", path, (long long)lineno);
    return GCNK_EARG;
  }
  std::fclose(f);
  // bounds first: a malformed or huge id must not size the allocation below
  if (maxid + 1 >= INT32_MAX || 2 * (int64_t)edges.size() >= INT32_MAX) {
    set_error("gcnk_edgelist: graph too large for int32 CSR (max id %lld, %lld edges)", (long long)maxid,
              (long long)edges.size());
    return GCNK_EUNSUP;
  }
  // distinct ids must be exactly 0..maxid
  std::vector<char> seen((size_t)(maxid + 1), 0);
  for (const Edge& e : edges) seen[(size_t)e.u] = seen[(size_t)e.v] = 1;
  for (int64_t i = 0; i <= maxid; ++i)
    if (!seen[(size_t)i]) {
      set_error("gcnk_edgelist: node ids are not contiguous (id %lld has no edge, max id %lld)", (long long)i,
                (long long)maxid);
      return GCNK_EUNSUP;
    }
  n = maxid + 1;
  // both directions; a repeated undirected edge keeps its last weight
  std::vector<Edge> both;
  both.reserve(edges.size() * 2);
  for (const Edge& e : edges) {
    both.push_back({e.u, e.v, e.order, e.w});
    if (e.u != e.v) both.push_back({e.v, e.u, e.order, e.w});
  }
  std::sort(both.begin(), both.end(), [](const Edge& a, const Edge& b) {
    return a.u != b.u ? a.u < b.u : (a.v != b.v ? a.v < b.v : a.order < b.order);
  });
  size_t o = 0;
  for (size_t i = 0; i < both.size(); ++i) {
    if (o > 0 && both[o - 1].u == both[i].u && both[o - 1].v == both[i].v) both[o - 1] = both[i];
    else both[o++] = both[i];
  }
  both.resize(o);
  edges.swap(both);
  return GCNK_OK;
}

// No exception may cross the extern "C" boundary: allocation failures become
// an error code.
int parse_guarded(const char* path, std::vector<Edge>& edges, int64_t& n) {
  try {
    return parse(path, edges, n);
  } catch (const std::exception& ex) {
    set_error("gcnk_edgelist: %s", ex.what());
    return GCNK_EUNSUP;
  }
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int gcnk_edgelist_size(const char* path, int64_t* n_nodes, int64_t* nnz) {
  if (!path || !n_nodes || !nnz) {
    set_error("gcnk_edgelist_size: null argument");
    return GCNK_EARG;
  }
  std::vector<Edge> e;
  int64_t n = 0;
  const int rc = parse_guarded(path, e, n);
  if (rc) return rc;
  *n_nodes = n;
  *nnz = (int64_t)e.size();
  return GCNK_OK;
}

extern "C" int gcnk_edgelist_csr(const char* path, int64_t n_nodes, int64_t nnz, int32_t* rowptr, int32_t* colind,
                                 float* val) {
  if (!path || !rowptr || (nnz > 0 && (!colind || !val))) {
    set_error("gcnk_edgelist_csr: null argument");
    return GCNK_EARG;
  }
  std::vector<Edge> e;
  int64_t n = 0;
  const int rc = parse_guarded(path, e, n);
  if (rc) return rc;
  if (n != n_nodes || (int64_t)e.size() != nnz) {
    set_error("gcnk_edgelist_csr: file has %lld nodes / %lld nonzeros, buffers sized for %lld / %lld", (long long)n,
              (long long)e.size(), (long long)n_nodes, (long long)nnz);
    return GCNK_EARG;
  }
  std::fill(rowptr, rowptr + n + 1, 0);
  for (size_t i = 0; i < e.size(); ++i) {
    ++rowptr[e[i].u + 1];
    colind[i] = (int32_t)e[i].v;
    val[i] = e[i].w;
  }
  for (int64_t r = 0; r < n; ++r) rowptr[r + 1] += rowptr[r];
  return GCNK_OK;
}
