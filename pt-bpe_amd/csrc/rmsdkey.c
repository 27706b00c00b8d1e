/* rmsdkey.c -- the pair key of the RMSD-partitioned mode (geobpe/rmsd_bpe.py RmsdBPE._pair_key),
 * the host hot spot of a step: the reference's compute_geo_key (foldingdiff/bpe.py:1192-1299)
 * reads a span's geometry (Tokenizer.token_geo, tokenizer.py:169-202), bins the items the pt1 /
 * pt2 rules select (bpe.py:1247-1285, get_ind :1164-1189) and renders
 * json.dumps(geo, sort_keys=True) (bpe.py:1147-1149), floats as Python's repr.
 *
 * A CPython extension so that it reads the chain's column lists in place (the host class keeps
 * them as Python lists; set_token_geo writes single cells).  Floats are formatted as
 * float.__repr__ does (frepr.cpp: std::to_chars' shortest digits in Python's layout) and
 * non-finite values as json does (NaN, Infinity, -Infinity).  A value outside the bins raises
 * the reference's ValueError with its message.
 *
 * key(cols, init, idx, l, ph, rng, thr) -> str
 *   cols  tuple of 9 column lists in ITEM order (below); init: list of 3 floats
 *   idx, l: the span (first bond, bonds); ph = idx % 3
 *   rng   ((lo, hi) per kind: bonds, angles, dihedrals) of the binned item indices
 *   thr   tuple of 9 (lefts, rights) float lists per item type, or None (type never binned)
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <string.h>

/* item types in json.dumps(sort_keys=True) order: name, kind (0 bond, 1 angle, 2 dihedral),
 * position of the type's first item within a residue (bpe.py's _ITEM) */
static const char* NAMES[9] = {"0C:1N", "C:1N:1CA", "CA:C", "CA:C:1N", "N:CA", "omega", "phi", "psi", "tau"};
static const int KIND[9] = {0, 1, 0, 1, 0, 2, 2, 2, 1};
static const int T0[9] = {2, 2, 1, 1, 0, 1, 2, 0, 0};
static const double TWO_PI = 6.283185307179586; /* 2 * np.pi */

typedef struct {
  char* p;
  Py_ssize_t n, cap;
} Buf;

static int buf_put(Buf* b, const char* s, Py_ssize_t n) {
  if (b->n + n > b->cap) {
    Py_ssize_t c = b->cap ? b->cap : 512;
    while (c < b->n + n) c *= 2;
    char* q = (char*)PyMem_Realloc(b->p, c);
    if (!q) {
      PyErr_NoMemory();
      return -1;
    }
    b->p = q;
    b->cap = c;
  }
  memcpy(b->p + b->n, s, n);
  b->n += n;
  return 0;
}
static int buf_str(Buf* b, const char* s) { return buf_put(b, s, (Py_ssize_t)strlen(s)); }

int geobpe_py_repr(double v, char* out); /* frepr.cpp: repr(float) from std::to_chars */

static int put_float(Buf* b, double v) {
  if (isnan(v)) return buf_str(b, "NaN");
  if (isinf(v)) return buf_str(b, v > 0 ? "Infinity" : "-Infinity");
  char s[40];
  return buf_put(b, s, geobpe_py_repr(v, s));
}

/* repr(float) of each value (the test of frepr.cpp against Python's own repr) */
static PyObject* reprs(PyObject* self, PyObject* args) {
  PyObject* vals;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!", &PyList_Type, &vals)) return NULL;
  PyObject* out = PyList_New(PyList_GET_SIZE(vals));
  if (!out) return NULL;
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(vals); i++) {
    const double v = PyFloat_AsDouble(PyList_GET_ITEM(vals, i));
    if (v == -1.0 && PyErr_Occurred()) {
      Py_DECREF(out);
      return NULL;
    }
    char s[40];
    PyList_SET_ITEM(out, i, PyUnicode_FromStringAndSize(s, geobpe_py_repr(v, s)));
  }
  return out;
}

/* Python's float % for a positive divisor (float_rem) */
static double py_mod(double x, double y) {
  double m = fmod(x, y);
  if (m) {
    if ((y < 0) != (m < 0)) m += y;
  } else {
    m = copysign(0.0, y);
  }
  return m;
}

/* BPE.get_ind (bpe.py:1164-1189): bisect_right over the left edges; -1 with ValueError set */
static long get_ind(double v, PyObject* lefts, PyObject* rights) {
  Py_ssize_t n = PyList_GET_SIZE(lefts), lo = 0, hi = n;
  while (lo < hi) { /* bisect_right */
    Py_ssize_t mid = (lo + hi) / 2;
    if (v < PyFloat_AS_DOUBLE(PyList_GET_ITEM(lefts, mid)))
      hi = mid;
    else
      lo = mid + 1;
  }
  Py_ssize_t ind = lo - 1;
  PyObject* fv;
  if (ind < 0) {
    fv = PyFloat_FromDouble(v);
    if (fv) {
      PyErr_Format(PyExc_ValueError, "value %R is below the first bin range", fv);
      Py_DECREF(fv);
    }
    return -1;
  }
  double a = PyFloat_AS_DOUBLE(PyList_GET_ITEM(lefts, ind)), b = PyFloat_AS_DOUBLE(PyList_GET_ITEM(rights, ind));
  if (ind == n - 1 && v == b) return (long)ind;
  if (a <= v && v < b) return (long)ind;
  fv = PyFloat_FromDouble(v);
  if (fv) {
    PyErr_Format(PyExc_ValueError, "value %R does not fall into any bin", fv);
    Py_DECREF(fv);
  }
  return -1;
}

static Py_ssize_t cnt_range(Py_ssize_t a, Py_ssize_t stop) { return a < stop ? (stop - a + 2) / 3 : 0; }
static Py_ssize_t floordiv3(Py_ssize_t x) { return x >= 0 ? x / 3 : -((-x + 2) / 3); }

/* value m of item type t of the span: token_geo's slices (init values in front of a column's rows) */
static int item_value(PyObject* cols, PyObject* init, int t, Py_ssize_t first, Py_ssize_t m, double* out) {
  PyObject* col = PyTuple_GET_ITEM(cols, t);
  Py_ssize_t row;
  const int kind = KIND[t];
  if (kind == 0) { /* bond j = first (< 2: init[j], then rows from 0) */
    if (first < 2) {
      if (m == 0) {
        *out = PyFloat_AsDouble(PyList_GET_ITEM(init, first));
        return 0;
      }
      row = m - 1;
    } else {
      row = (first - 2) / 3 + m;
    }
  } else if (kind == 1) { /* angle a = first (0: init[2]) */
    if (first == 0) {
      if (m == 0) {
        *out = PyFloat_AsDouble(PyList_GET_ITEM(init, 2));
        return 0;
      }
      row = m - 1;
    } else {
      row = (first - 1) / 3 + m;
    }
  } else {
    row = (first + 1) / 3 + m;
  }
  if (row < 0 || row >= PyList_GET_SIZE(col)) {
    PyErr_SetString(PyExc_IndexError, "rmsdkey: span outside the chain");
    return -1;
  }
  *out = PyFloat_AsDouble(PyList_GET_ITEM(col, row));
  return PyErr_Occurred() ? -1 : 0;
}

static PyObject* key(PyObject* self, PyObject* args) {
  PyObject *cols, *init, *rng, *thr;
  Py_ssize_t idx, l, ph;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!nnnO!O!", &PyTuple_Type, &cols, &PyList_Type, &init, &idx, &l, &ph, &PyTuple_Type,
                        &rng, &PyTuple_Type, &thr))
    return NULL;
  if (PyTuple_GET_SIZE(cols) != 9 || PyTuple_GET_SIZE(thr) != 9 || PyTuple_GET_SIZE(rng) != 3 ||
      PyList_GET_SIZE(init) < 3) {
    PyErr_SetString(PyExc_ValueError, "rmsdkey.key: bad argument shapes");
    return NULL;
  }
  for (int t = 0; t < 9; t++)
    if (!PyList_Check(PyTuple_GET_ITEM(cols, t))) {
      PyErr_SetString(PyExc_TypeError, "rmsdkey.key: columns must be lists");
      return NULL;
    }
  Py_ssize_t lo[3], hi[3];
  for (int k = 0; k < 3; k++) {
    PyObject* p = PyTuple_GET_ITEM(rng, k);
    if (!PyArg_ParseTuple(p, "nn", &lo[k], &hi[k])) return NULL;
  }
  Buf b = {NULL, 0, 0};
  int first_key = 1;
  char num[32];
  if (buf_str(&b, "{") < 0) goto fail;
  for (int t = 0; t < 9; t++) {
    const int kind = KIND[t];
    /* the type's first item in the span and its count (token_geo: bonds over l, angles over
       l - 1, dihedrals over l - 2 items; type j % 3 of the first three) */
    const Py_ssize_t nitems = kind == 0 ? l : (kind == 1 ? l - 1 : l - 2);
    Py_ssize_t first = -1;
    for (Py_ssize_t j = idx; j < idx + (nitems < 3 ? nitems : 3); j++) {
      const int tt = kind == 0 ? (int)(j % 3) : (int)(j % 3);
      /* type of item j: BOND_TYPES / BOND_ANGLES / DIHEDRALS [j % 3] */
      static const int BT[3] = {4, 2, 0}, BA[3] = {8, 3, 1}, DH[3] = {7, 5, 6};
      const int ty = kind == 0 ? BT[tt] : (kind == 1 ? BA[tt] : DH[tt]);
      if (ty == t) {
        first = j;
        break;
      }
    }
    if (first < 0) continue;
    const Py_ssize_t cnt = cnt_range(first, idx + nitems);
    /* binned items m in [m_lo, m_hi): base + 3m in [lo, hi), base = (t0 + 3 - ph) % 3 */
    const Py_ssize_t base = (T0[t] + 3 - ph) % 3;
    Py_ssize_t m_lo = 0, m_hi = 0;
    if (lo[kind] < hi[kind]) {
      m_lo = -floordiv3(base - lo[kind]);
      if (m_lo < 0) m_lo = 0;
      m_hi = -floordiv3(base - hi[kind]);
      if (m_hi > cnt) m_hi = cnt;
    }
    PyObject* th = PyTuple_GET_ITEM(thr, t);
    if (m_lo < m_hi && (th == Py_None || !PyTuple_Check(th) || PyTuple_GET_SIZE(th) != 2)) {
      PyErr_SetString(PyExc_ValueError, "rmsdkey.key: no thresholds for a binned item type");
      goto fail;
    }
    if (!first_key && buf_str(&b, ", ") < 0) goto fail;
    first_key = 0;
    if (buf_str(&b, "\"") < 0 || buf_str(&b, NAMES[t]) < 0 || buf_str(&b, "\": [") < 0) goto fail;
    for (Py_ssize_t m = 0; m < cnt; m++) {
      double v;
      if (item_value(cols, init, t, first, m, &v) < 0) goto fail;
      if (m && buf_str(&b, ", ") < 0) goto fail;
      if (m >= m_lo && m < m_hi) {
        const double q = kind == 0 ? v : py_mod(v + TWO_PI, TWO_PI);
        const long ind = get_ind(q, PyTuple_GET_ITEM(th, 0), PyTuple_GET_ITEM(th, 1));
        if (ind < 0) goto fail;
        snprintf(num, sizeof num, "%ld", ind);
        if (buf_str(&b, num) < 0) goto fail;
      } else if (put_float(&b, v) < 0) {
        goto fail;
      }
    }
    if (buf_str(&b, "]") < 0) goto fail;
  }
  if (buf_str(&b, "}") < 0) goto fail;
  PyObject* out = PyUnicode_FromStringAndSize(b.p, b.n);
  PyMem_Free(b.p);
  return out;
fail:
  PyMem_Free(b.p);
  return NULL;
}

/* pack(spans, out) -- the whole-residue geometry of many spans in geobpe_nerf's layout
 * (9 float64 per residue: N:CA, CA:C, tau, 0C:1N, CA:C:1N, C:1N:1CA, psi, omega, phi; the last
 * residue of a span only its first three), the token_geo of Tokenizer.compute_coords
 * (tokenizer.py:347-363) without the dicts.  spans: list of (cols, init, q, r) -- the chain's
 * nine column lists in that order, its init triple, the first residue q and the residues r;
 * out: a writable C-contiguous float64 buffer of sum(r) * 9.  Residue q + k reads row
 * q + k - 1 of N:CA / CA:C / tau (residue 0: init) and row q + k of the junction columns
 * (phi: row q + k + 1) -- bond j -> row (j - 2) // 3, angle a -> (a - 1) // 3, dihedral d ->
 * (d + 1) // 3 (rmsd_bpe._Chain). */
static PyObject* pack(PyObject* self, PyObject* args) {
  PyObject* spans;
  Py_buffer out;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!w*", &PyList_Type, &spans, &out)) return NULL;
  double* o = (double*)out.buf;
  const Py_ssize_t cap = out.len / (Py_ssize_t)sizeof(double);
  Py_ssize_t at = 0;
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(spans); i++) {
    PyObject *cols, *init;
    Py_ssize_t q, r;
    if (!PyArg_ParseTuple(PyList_GET_ITEM(spans, i), "O!O!nn", &PyTuple_Type, &cols, &PyList_Type, &init, &q, &r))
      goto fail;
    if (PyTuple_GET_SIZE(cols) != 9 || PyList_GET_SIZE(init) < 3 || q < 0 || r < 1 || at + 9 * r > cap) {
      PyErr_SetString(PyExc_ValueError, "rmsdkey.pack: bad span");
      goto fail;
    }
    for (Py_ssize_t k = 0; k < r; k++, at += 9) {
      const Py_ssize_t res = q + k;
      for (int c = 0; c < 9; c++) {
        double v = 0.0;
        if (c < 3) {
          if (res == 0) {
            v = PyFloat_AsDouble(PyList_GET_ITEM(init, c));
          } else {
            PyObject* col = PyTuple_GET_ITEM(cols, c);
            if (res - 1 >= PyList_GET_SIZE(col)) goto range;
            v = PyFloat_AsDouble(PyList_GET_ITEM(col, res - 1));
          }
        } else if (k + 1 < r) {
          PyObject* col = PyTuple_GET_ITEM(cols, c);
          const Py_ssize_t row = c == 8 ? res + 1 : res;
          if (row >= PyList_GET_SIZE(col)) goto range;
          v = PyFloat_AsDouble(PyList_GET_ITEM(col, row));
        }
        if (v == -1.0 && PyErr_Occurred()) goto fail;
        o[at + c] = v;
      }
    }
  }
  PyBuffer_Release(&out);
  return PyLong_FromSsize_t(at / 9);
range:
  PyErr_SetString(PyExc_IndexError, "rmsdkey.pack: span outside the chain");
fail:
  PyBuffer_Release(&out);
  return NULL;
}

/* setgeo(cols, init, idx, l, vals) -> bool -- Tokenizer.set_token_geo (tokenizer.py:253-286) as
 * the host class does it (rmsd_bpe._Chain.set_geo): the span's bonds, angles and dihedrals take
 * vals[type]'s items in order (the same objects), bond 0/1 and angle 0 going to init.  cols: the
 * nine column lists in json key order (as key()).  Returns False, having written nothing, when
 * a type is missing, too short or has items left over: the Python version then raises the
 * reference's error. */
static PyObject* setgeo(PyObject* self, PyObject* args) {
  PyObject *cols, *init, *vals;
  Py_ssize_t idx, l;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!nnO!", &PyTuple_Type, &cols, &PyList_Type, &init, &idx, &l, &PyDict_Type, &vals))
    return NULL;
  if (PyTuple_GET_SIZE(cols) != 9 || PyList_GET_SIZE(init) < 3 || idx < 0 || l < 1) {
    PyErr_SetString(PyExc_ValueError, "rmsdkey.setgeo: bad arguments");
    return NULL;
  }
  static const int BT[3] = {4, 2, 0}, BA[3] = {8, 3, 1}, DH[3] = {7, 5, 6};
  PyObject* seq[9] = {NULL};
  Py_ssize_t need[9] = {0}, pos[9] = {0};
  for (Py_ssize_t j = idx; j < idx + l; j++) need[BT[j % 3]]++;
  for (Py_ssize_t j = idx; j < idx + l - 1; j++) need[BA[j % 3]]++;
  for (Py_ssize_t j = idx; j < idx + l - 2; j++) need[DH[j % 3]]++;
  PyObject* ok = Py_True;
  /* every type in vals must be used up exactly; every needed type present and long enough */
  PyObject *k, *v;
  Py_ssize_t it = 0;
  while (PyDict_Next(vals, &it, &k, &v)) {
    int t = -1;
    for (int q = 0; q < 9; q++)
      if (PyUnicode_Check(k) && PyUnicode_CompareWithASCIIString(k, NAMES[q]) == 0) t = q;
    if (t < 0) {
      ok = Py_False;
      break;
    }
    PyObject* f = PySequence_Fast(v, "rmsdkey.setgeo: values must be sequences");
    if (!f) goto fail;
    seq[t] = f;
    if (PySequence_Fast_GET_SIZE(f) != need[t]) ok = Py_False;
  }
  for (int t = 0; t < 9 && ok == Py_True; t++)
    if (need[t] > 0 && !seq[t]) ok = Py_False;
  if (ok == Py_True) {
    /* bounds first (Python would raise IndexError midway): all rows inside their columns */
    for (Py_ssize_t j = idx; j < idx + l && ok == Py_True; j++)
      if (j >= 2 && (j - 2) / 3 >= PyList_GET_SIZE(PyTuple_GET_ITEM(cols, BT[j % 3]))) ok = Py_False;
    for (Py_ssize_t j = idx; j < idx + l - 1 && ok == Py_True; j++)
      if (j >= 1 && (j - 1) / 3 >= PyList_GET_SIZE(PyTuple_GET_ITEM(cols, BA[j % 3]))) ok = Py_False;
    for (Py_ssize_t j = idx; j < idx + l - 2 && ok == Py_True; j++)
      if ((j + 1) / 3 >= PyList_GET_SIZE(PyTuple_GET_ITEM(cols, DH[j % 3]))) ok = Py_False;
  }
  if (ok == Py_True) {
#define SETGEO_PUT(LIST, ROW, T)                                     \
  do {                                                              \
    PyObject* x_ = PySequence_Fast_GET_ITEM(seq[T], pos[T]++);      \
    Py_INCREF(x_);                                                  \
    PyList_SetItem((LIST), (ROW), x_);                              \
  } while (0)
    for (Py_ssize_t j = idx; j < idx + l; j++) {
      const int t = BT[j % 3];
      if (j < 2)
        SETGEO_PUT(init, j, t);
      else
        SETGEO_PUT(PyTuple_GET_ITEM(cols, t), (j - 2) / 3, t);
    }
    for (Py_ssize_t j = idx; j < idx + l - 1; j++) {
      const int t = BA[j % 3];
      if (j == 0)
        SETGEO_PUT(init, 2, t);
      else
        SETGEO_PUT(PyTuple_GET_ITEM(cols, t), (j - 1) / 3, t);
    }
    for (Py_ssize_t j = idx; j < idx + l - 2; j++) {
      const int t = DH[j % 3];
      SETGEO_PUT(PyTuple_GET_ITEM(cols, t), (j + 1) / 3, t);
    }
#undef SETGEO_PUT
  }
  for (int t = 0; t < 9; t++) Py_XDECREF(seq[t]);
  Py_INCREF(ok);
  return ok;
fail:
  for (int t = 0; t < 9; t++) Py_XDECREF(seq[t]);
  return NULL;
}

static PyMethodDef METHODS[] = {{"key", key, METH_VARARGS, "the pair key string of a span (RmsdBPE._pair_key)"},
                                {"pack", pack, METH_VARARGS, "whole-residue span geometry, geobpe_nerf layout"},
                                {"reprs", reprs, METH_VARARGS, "repr(float) of each value (test)"},
                                {"setgeo", setgeo, METH_VARARGS, "set_token_geo into the chain's column lists"},
                                {NULL, NULL, 0, NULL}};
static struct PyModuleDef MOD = {PyModuleDef_HEAD_INIT, "_rmsdkey", NULL, -1, METHODS, NULL, NULL, NULL, NULL};
PyMODINIT_FUNC PyInit__rmsdkey(void) { return PyModule_Create(&MOD); }
