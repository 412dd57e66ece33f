// glm.hpp -- the least-squares "logistic" classifier fit of MeShClust's Trainer.
//
// Restates matrix::Matrix (src/cluster/src/Matrix.cpp) and matrix::GLM
// (src/cluster/src/GLM.cpp) with the reference build's exact floating-point operation
// order: Matrix::operator* accumulates with a fused multiply-add (vfmadd231sd in the
// reference object) and the Gauss-Jordan row updates are fused negative multiply-adds
// (vfnmadd231sd/132sd).  This file is compiled with -ffp-contract=off so that only the
// explicit std::fma calls fuse.  The fit is tiny (<= 5 columns x ~3,000 rows): host-side.
#pragma once
#include <cstddef>
#include <tuple>
#include <vector>

namespace mc {

struct Matrix {
  int rows = 0, cols = 0;
  std::vector<double> m;  // row-major
  Matrix() = default;
  Matrix(int r, int c) : rows(r), cols(c), m((size_t)r * c, 0.0) {}
  double get(int r, int c) const { return m[(size_t)r * cols + c]; }
  void set(int r, int c, double v) { m[(size_t)r * cols + c] = v; }
  Matrix transpose() const;
  Matrix mul(const Matrix &n) const;   // Matrix::operator* (Matrix.cpp:69-89)
  Matrix gauss_jordan_inverse();       // Matrix.cpp:102-200
  Matrix pseudo_inverse() const;       // Matrix.cpp:202-214
};

struct GLM {
  Matrix weights;
  void train(const Matrix &features, const Matrix &labels);  // GLM.cpp:19-22
  Matrix predict(const Matrix &features) const;              // GLM.cpp:24-33
  // GLM.cpp:35-63 (prints like the reference when verbose)
  std::tuple<double, double, double> accuracy(const Matrix &o, const Matrix &p, bool verbose) const;
};

}  // namespace mc
