// =====================================================================================
//  oracle/or_match.cpp  --  TEST INFRASTRUCTURE ONLY (parity vs real PCL UNPINNED)
//
//  CPU restatement of the reference's descriptor matching:
//    Features<T>::getCorrespondences   include/pcl_feature_extraction/features.h:255-273
//    Features<T>::findCorrespondences  include/pcl_feature_extraction/features.h:224-253
//  i.e. for every source descriptor the 1-nearest target descriptor through
//  pcl::KdTreeFLANN<FeatureT> (FLANN 1.8 KDTreeSingleIndex, exact search: max checks -1,
//  eps 0), in both directions, then the mutual check target2source[source2target[i]] == i.
//
//  Arithmetic restated (FLANN dist.h L2_Simple<float>, the default Dist of KdTreeFLANN):
//    d(a, b) = sequential float sum over dims 0..D-1 of (a_k - b_k)^2, no FMA.
//  Index contents (PCL kdtree_flann.hpp convertCloudToArray): rows with a non-finite value
//  are not indexed (DefaultFeatureRepresentation::isValid); returned indices are cloud rows.
//  Restatement choices (documented in DESIGN.md, unpinned):
//    * ties (equal float distance): the lowest target row wins.  FLANN keeps the first
//      point visited (KNNSimpleResultSet::addPoint rejects dist >= worst), i.e. the kd-tree
//      traversal order, which depends on the tree build;
//    * a non-finite source row has no match (-1).  In the reference this is undefined:
//      FLANN 1.8.4 copies an uninitialised index when no finite distance exists;
//    * a target without any finite row: every source row has no match (the reference
//      indexes k_indices[0] of an empty vector).
// =====================================================================================
#include <cmath>
#include <cstdint>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

typedef int64_t i64;

namespace {

bool finiteRow(const float* r, int dim) {
  for (int k = 0; k < dim; ++k)
    if (!std::isfinite(r[k])) return false;
  return true;
}

// flann::L2_Simple<float>::operator()
inline float l2Simple(const float* a, const float* b, int dim) {
  float result = 0.0f;
  for (int k = 0; k < dim; ++k) {
    const float diff = a[k] - b[k];
    result += diff * diff;
  }
  return result;
}

// Features::getCorrespondences: source2target[i] (and the matched squared distance)
void nearest(const float* src, i64 ns, const float* tgt, i64 nt, int dim, int32_t* idx, float* dist,
             int threads) {
  std::vector<char> valid((size_t)nt);
  for (i64 j = 0; j < nt; ++j) valid[(size_t)j] = finiteRow(tgt + j * dim, dim);
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
  for (i64 i = 0; i < ns; ++i) {
    const float* a = src + i * dim;
    int32_t best = -1;
    float bd = 0.0f;
    if (finiteRow(a, dim)) {
      for (i64 j = 0; j < nt; ++j) {
        if (!valid[(size_t)j]) continue;
        const float d = l2Simple(a, tgt + j * dim, dim);
        if (best < 0 || d < bd) {  // strict: the lowest row keeps a tie
          best = (int32_t)j;
          bd = d;
        }
      }
    }
    idx[i] = best;
    if (dist) dist[i] = best >= 0 ? bd : NAN;
  }
}

}  // namespace

extern "C" {

int orc_nearest_descriptor(const float* src, i64 ns, const float* tgt, i64 nt, int dim, int32_t* idx,
                           float* dist, int threads) {
  if (ns < 0 || nt < 0 || dim <= 0) return 1;
  nearest(src, ns, tgt, nt, dim, idx, dist, threads);
  return 0;
}

// Features::findCorrespondences: (index_query, index_match) pairs in source order.
int orc_correspondences(const float* src, i64 ns, const float* tgt, i64 nt, int dim, int32_t* query,
                        int32_t* match, i64 cap, i64* n_out, int threads) {
  if (ns < 0 || nt < 0 || dim <= 0) return 1;
  std::vector<int32_t> s2t((size_t)ns), t2s((size_t)nt);
  nearest(src, ns, tgt, nt, dim, s2t.data(), nullptr, threads);
  nearest(tgt, nt, src, ns, dim, t2s.data(), nullptr, threads);
  i64 n = 0;
  for (i64 c = 0; c < ns; ++c) {
    const int32_t m = s2t[(size_t)c];
    if (m >= 0 && t2s[(size_t)m] == c) {
      if (n < cap) {
        query[n] = (int32_t)c;
        match[n] = m;
      }
      ++n;
    }
  }
  *n_out = n;
  return n > cap ? 3 : 0;
}

}  // extern "C"
