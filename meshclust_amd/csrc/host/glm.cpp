// glm.cpp -- see glm.hpp.  Compiled with -ffp-contract=off.
#include "glm.hpp"

#include <cmath>
#include <cstdio>

#include "common.hpp"

namespace mc {

Matrix Matrix::transpose() const {
  Matrix t(cols, rows);
  for (int i = 0; i < rows; i++)
    for (int j = 0; j < cols; j++) t.set(j, i, get(i, j));
  return t;
}

Matrix Matrix::mul(const Matrix &n) const {
  if (cols != n.rows) throw Error("Invalid input: array dimension mismatch.", 1);
  Matrix r(rows, n.cols);
  for (int i = 0; i < rows; i++)
    for (int j = 0; j < n.cols; j++) {
      double cur = 0;
      for (int k = 0; k < cols; k++) cur = std::fma(get(i, k), n.get(k, j), cur);
      r.set(i, j, cur);
    }
  return r;
}

// Gauss-Jordan with the reference's pivot rules: divide the pivot row when the pivot is
// not exactly 1, swap with the first lower row holding a non-zero when it is 0, then
// eliminate below and (afterwards, bottom-up) above.  On failure the reference prints and
// returns the ORIGINAL matrix (Matrix.cpp:143-147, 181-193).
Matrix Matrix::gauss_jordan_inverse() {
  if (rows != cols) throw Error("Invalid dimensions", 1);
  const int n = rows;
  Matrix inv(n, n);
  Matrix saved = *this;
  for (int i = 0; i < n; i++) inv.set(i, i, 1);
  for (int i = 0; i < n; i++) {
    if (get(i, i) != 1) {
      if (get(i, i) != 0) {
        double pv = get(i, i);
        for (int j = 0; j < n; j++) {
          set(i, j, get(i, j) / pv);
          inv.set(i, j, inv.get(i, j) / pv);
        }
      } else {
        int row = i + 1;
        bool ok = false;
        while (!ok && row < n) {
          if (get(row, i) != 0) ok = true;
          else row++;
        }
        if (!ok) {
          printf("Inverse does not exist\n");
          *this = saved;
          return saved;
        }
        for (int j = 0; j < n; j++) {
          double a = get(i, j), b = inv.get(i, j);
          set(i, j, get(row, j));
          inv.set(i, j, inv.get(row, j));
          set(row, j, a);
          inv.set(row, j, b);
        }
        double pv = get(i, i);
        for (int j = 0; j < n; j++) {
          set(i, j, get(i, j) / pv);
          inv.set(i, j, inv.get(i, j) / pv);
        }
      }
    }
    for (int below = i + 1; below < n; below++) {
      if (get(below, i) != 0) {
        double pv = get(below, i);
        for (int j = 0; j < n; j++) {
          set(below, j, std::fma(-pv, get(i, j), get(below, j)));
          inv.set(below, j, std::fma(-pv, inv.get(i, j), inv.get(below, j)));
        }
      }
    }
  }
  for (int i = n - 1; i >= 0; i--) {
    for (int above = 0; above < i; above++) {
      if (get(above, i) != 0) {
        double pv = get(above, i);
        for (int j = 0; j < n; j++) {
          set(above, j, std::fma(-pv, get(i, j), get(above, j)));
          inv.set(above, j, std::fma(-pv, inv.get(i, j), inv.get(above, j)));
        }
      }
    }
  }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      if ((i == j && get(i, j) != 1) || (i != j && get(i, j) != 0)) {
        printf("Inverse does not exist\n");
        *this = saved;
        return saved;
      }
    }
  *this = saved;
  return inv;
}

Matrix Matrix::pseudo_inverse() const {
  if (rows >= cols) {
    Matrix t = transpose();
    Matrix tbo = t.mul(*this);
    return tbo.gauss_jordan_inverse().mul(t);
  }
  Matrix t = transpose();
  Matrix obt = mul(t);
  return t.mul(obt.gauss_jordan_inverse());
}

void GLM::train(const Matrix &features, const Matrix &labels) {
  Matrix ft = features.transpose();
  Matrix w = ft.mul(features);
  // weights.pseudoInverse() * features.transpose() * labels, evaluated left to right
  weights = w.pseudo_inverse().mul(features.transpose()).mul(labels);
}

Matrix GLM::predict(const Matrix &features) const {
  Matrix labels = features.mul(weights);
  for (int i = 0; i < labels.rows; i++) labels.set(i, 0, std::round(1 / (1 + std::exp(-(labels.get(i, 0))))));
  return labels;
}

std::tuple<double, double, double> GLM::accuracy(const Matrix &o, const Matrix &p, bool verbose) const {
  int sum = 0, negSum = 0, negSame = 0, posSum = 0, posSame = 0;
  for (int i = 0; i < o.rows; i++) {
    if (o.get(i, 0) == -1) {
      negSum++;
      if (o.get(i, 0) == p.get(i, 0)) { sum++; negSame++; }
    } else {
      posSum++;
      if (o.get(i, 0) == p.get(i, 0)) { sum++; posSame++; }
    }
  }
  double acc = ((double)sum * 100) / (o.rows);
  double sens = ((double)posSame * 100) / (posSum);
  double spec = ((double)negSame * 100) / (negSum);
  if (verbose) printf("Accuracy: %g%% Sensitivity: %g%% Specificity: %g%% \n", acc, sens, spec);
  return std::make_tuple(acc, sens, spec);
}

}  // namespace mc
