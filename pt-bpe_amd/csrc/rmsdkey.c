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

/* attribute and column names, interned once at import (the ...String() lookups built and
 * hashed a new str per call, ~10 per chain visited) */
enum { A_CUR, A_ORIG, A_INIT, A_TOKEN_POS, A_BTT, A_EVENTS, A_N, A_COUNT };
static const char* ATTR_NAMES[A_COUNT] = {"cur", "orig", "init", "token_pos", "btt", "events", "n"};
/* RMSDKEY_PROF=1 (a profiling build): nanoseconds per section of merge(), read by prof() */
#define PROF_T(v)
#define PROF_ADD(i, t0)

static PyObject* ATTR[A_COUNT];
static PyObject* PACK_KEYS[9];
static PyObject* NAME_KEYS[9]; /* NAMES interned: a struc dict's keys are found by identity first */

typedef struct {
  char* p;
  Py_ssize_t n, cap;
  char* stack; /* p's first buffer (the caller's); grown on the heap */
} Buf;

static int buf_put(Buf* b, const char* s, Py_ssize_t n) {
  if (b->n + n > b->cap) {
    Py_ssize_t c = b->cap ? b->cap : 512;
    while (c < b->n + n) c *= 2;
    char* q = (char*)PyMem_Malloc(c);
    if (!q) {
      PyErr_NoMemory();
      return -1;
    }
    memcpy(q, b->p, b->n);
    if (b->p != b->stack) PyMem_Free(b->p);
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

static PyObject* build_key(PyObject* cols, PyObject* init, Py_ssize_t idx, Py_ssize_t l, Py_ssize_t ph,
                           const Py_ssize_t* lo, const Py_ssize_t* hi, PyObject* thr);

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
  return build_key(cols, init, idx, l, ph, lo, hi, thr);
}

/* the span's value objects, fetched ahead: a key reads ~25 floats scattered over the heap, and
 * one after the other each was a dependent cache miss */
static void prefetch_span(PyObject* cols, Py_ssize_t idx, Py_ssize_t l) {
  static const int BT[3] = {4, 2, 0}, BA[3] = {8, 3, 1}, DH[3] = {7, 5, 6};
  for (Py_ssize_t j = idx > 2 ? idx : 2; j < idx + l; j++) {
    PyObject* col = PyTuple_GET_ITEM(cols, BT[j % 3]);
    const Py_ssize_t row = (j - 2) / 3;
    if (row < PyList_GET_SIZE(col)) __builtin_prefetch(PyList_GET_ITEM(col, row));
  }
  for (Py_ssize_t j = idx > 1 ? idx : 1; j < idx + l - 1; j++) {
    PyObject* col = PyTuple_GET_ITEM(cols, BA[j % 3]);
    const Py_ssize_t row = (j - 1) / 3;
    if (row < PyList_GET_SIZE(col)) __builtin_prefetch(PyList_GET_ITEM(col, row));
  }
  for (Py_ssize_t j = idx; j < idx + l - 2; j++) {
    PyObject* col = PyTuple_GET_ITEM(cols, DH[j % 3]);
    const Py_ssize_t row = (j + 1) / 3;
    if (row < PyList_GET_SIZE(col)) __builtin_prefetch(PyList_GET_ITEM(col, row));
  }
}

static PyObject* build_key(PyObject* cols, PyObject* init, Py_ssize_t idx, Py_ssize_t l, Py_ssize_t ph,
                           const Py_ssize_t* lo, const Py_ssize_t* hi, PyObject* thr) {
  prefetch_span(cols, idx, l);
  char stack[2048];
  Buf b = {stack, 0, (Py_ssize_t)sizeof stack, stack};
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
    if (m_lo < m_hi && (!PyTuple_Check(th) || PyTuple_GET_SIZE(th) != 2)) {
      /* the type has no thresholds at this length: _edges_for stored the exception the
         reference's lookup raised (KeyError / TypeError, bpe.py:1247-1296); raise that one */
      if (PyExceptionInstance_Check(th))
        PyErr_SetObject((PyObject*)Py_TYPE(th), th);
      else
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
        int k = (int)sizeof num;  /* (the bin index in decimal: snprintf cost more than the rest of a key) */
        long x = ind;
        do {
          num[--k] = (char)('0' + x % 10);
          x /= 10;
        } while (x);
        if (buf_put(&b, num + k, (Py_ssize_t)sizeof num - k) < 0) goto fail;
      } else if (put_float(&b, v) < 0) {
        goto fail;
      }
    }
    if (buf_str(&b, "]") < 0) goto fail;
  }
  if (buf_str(&b, "}") < 0) goto fail;
  PROF_T(uk0);
  PyObject* out = PyUnicode_New(b.n, 127);  /* (every character is ASCII) */
  if (out) memcpy(PyUnicode_DATA(out), b.p, b.n);
  PROF_ADD(7, uk0);
  if (b.p != stack) PyMem_Free(b.p);
  return out;
fail:
  if (b.p != stack) PyMem_Free(b.p);
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
/* one span into o[9 r]: 0, -1 with IndexError (outside the chain) or another error set */
static int pack_one(PyObject* cols, PyObject* init, Py_ssize_t q, Py_ssize_t r, double* o) {
  for (int c = 0; c < 9; c++) {  /* (the value objects first: each read is a cache miss) */
    PyObject* col = PyTuple_GET_ITEM(cols, c);
    const Py_ssize_t n = PyList_GET_SIZE(col);
    for (Py_ssize_t k = 0; k < r; k++) {
      const Py_ssize_t row = c < 3 ? q + k - 1 : (k + 1 < r ? (c == 8 ? q + k + 1 : q + k) : -1);
      if (row >= 0 && row < n) __builtin_prefetch(PyList_GET_ITEM(col, row));
    }
  }
  for (Py_ssize_t k = 0; k < r; k++, o += 9) {
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
      if (v == -1.0 && PyErr_Occurred()) return -1;
      o[c] = v;
    }
  }
  return 0;
range:
  PyErr_SetString(PyExc_IndexError, "rmsdkey.pack: span outside the chain");
  return -1;
}

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
    for (int c = 0; c < 9; c++)
      if (!PyList_Check(PyTuple_GET_ITEM(cols, c))) {
        PyErr_SetString(PyExc_TypeError, "rmsdkey.pack: columns must be lists");
        goto fail;
      }
    if (pack_one(cols, init, q, r, o + at) < 0) goto fail;
    at += 9 * r;
  }
  PyBuffer_Release(&out);
  return PyLong_FromSsize_t(at / 9);
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
/* 1: written; 0: does not fit (nothing written); -1: error set */
static int setgeo_impl(PyObject* cols, PyObject* init, Py_ssize_t idx, Py_ssize_t l, PyObject* vals) {
  if (PyTuple_GET_SIZE(cols) != 9 || PyList_GET_SIZE(init) < 3 || idx < 0 || l < 1) {
    PyErr_SetString(PyExc_ValueError, "rmsdkey.setgeo: bad arguments");
    return -1;
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
    for (int q = 0; q < 9 && t < 0; q++)
      if (k == NAME_KEYS[q]) t = q;
    for (int q = 0; q < 9 && t < 0; q++)
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
/* (a cell that already holds the very object is left alone: a partitioned token's medoid
   geometry is mostly its parts' medoid values, the objects the span already holds) */
#define SETGEO_PUT(LIST, ROW, T)                                     \
  do {                                                              \
    PyObject* x_ = PySequence_Fast_GET_ITEM(seq[T], pos[T]++);      \
    if (PyList_GET_ITEM((LIST), (ROW)) != x_) {                     \
      Py_INCREF(x_);                                                \
      PyList_SetItem((LIST), (ROW), x_);                            \
    }                                                               \
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
  return ok == Py_True ? 1 : 0;
fail:
  for (int t = 0; t < 9; t++) Py_XDECREF(seq[t]);
  return -1;
}

static PyObject* setgeo(PyObject* self, PyObject* args) {
  PyObject *cols, *init, *vals;
  Py_ssize_t idx, l;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!nnO!", &PyTuple_Type, &cols, &PyList_Type, &init, &idx, &l, &PyDict_Type, &vals))
    return NULL;
  const int rc = setgeo_impl(cols, init, idx, l, vals);
  if (rc < 0) return NULL;
  return PyBool_FromLong(rc);
}

/* ---------------------------------------------------------------- the merge loop
 * merge(st, occs, assigns, key, length, n, rmsd, vals, diff) -- the occurrence loop of
 * BPE.step (bpe.py:1860-2013) as RmsdBPE._merge runs it (without the multi-grid stale-key
 * path), on the host class's own objects: the same Python sets, dicts and lists are changed
 * in the same order, so every later list(set) (the order k-medoids sees) is CPython's.
 *   st      (chains, gd, pk, edges, edges_fn, names): the _Chain list, _geo_dict
 *           (defaultdict(set)), _pk, the per-length threshold edges and the callable that
 *           makes a missing length's, the column names in json key order
 *   occs    the occurrences (ci, i2) in sorted order; assigns: their medoids (rmsd) or None
 *   vals    rmsd: the medoid geometries of the key; else the binned geometry
 *   diff    note(): key -> count change                                                  */
/* The pair-key memo (mpair_key): an open-addressing table of 9-word signatures -> key str,
 * owned by a capsule per RmsdBPE instance (a Python dict keyed by bytes cost an allocation
 * and a 72-byte hash per lookup) */
typedef struct {
  long long w[9];
  PyObject* v; /* NULL: empty */
} MemoEnt;
typedef struct {
  Py_ssize_t n, cap; /* cap: a power of two */
  MemoEnt* e;
} Memo;
static const char* MEMO_NAME = "rmsdkey.memo";

static void memo_destroy(PyObject* capsule) {
  Memo* m = (Memo*)PyCapsule_GetPointer(capsule, MEMO_NAME);
  if (!m) return;
  for (Py_ssize_t i = 0; i < m->cap; i++) Py_XDECREF(m->e[i].v);
  PyMem_Free(m->e);
  PyMem_Free(m);
}
static PyObject* memo_new(PyObject* self, PyObject* noargs) {
  (void)self;
  (void)noargs;
  Memo* m = (Memo*)PyMem_Calloc(1, sizeof(Memo));
  if (!m) return PyErr_NoMemory();
  m->cap = 1 << 12;
  m->e = (MemoEnt*)PyMem_Calloc((size_t)m->cap, sizeof(MemoEnt));
  if (!m->e) {
    PyMem_Free(m);
    return PyErr_NoMemory();
  }
  PyObject* c = PyCapsule_New(m, MEMO_NAME, memo_destroy);
  if (!c) {
    PyMem_Free(m->e);
    PyMem_Free(m);
  }
  return c;
}
static PyObject* memo_len(PyObject* self, PyObject* capsule) {
  (void)self;
  Memo* m = (Memo*)PyCapsule_GetPointer(capsule, MEMO_NAME);
  return m ? PyLong_FromSsize_t(m->n) : NULL;
}
static unsigned long long memo_hash(const long long* w) {
  unsigned long long h = 0x9E3779B97F4A7C15ULL;
  for (int i = 0; i < 9; i++) {
    h ^= (unsigned long long)w[i];
    h *= 0xBF58476D1CE4E5B9ULL;
    h ^= h >> 31;
  }
  return h;
}
static MemoEnt* memo_slot(Memo* m, const long long* w) { /* the entry holding w, or the empty one it goes to */
  Py_ssize_t i = (Py_ssize_t)(memo_hash(w) & (unsigned long long)(m->cap - 1));
  for (;;) {
    MemoEnt* e = &m->e[i];
    if (!e->v || memcmp(e->w, w, sizeof e->w) == 0) return e;
    i = (i + 1) & (m->cap - 1);
  }
}
static int memo_put(Memo* m, const long long* w, PyObject* v) {
  if (2 * (m->n + 1) > m->cap) { /* grow to keep the load under 1/2 */
    Memo big = {0, 2 * m->cap, (MemoEnt*)PyMem_Calloc((size_t)(2 * m->cap), sizeof(MemoEnt))};
    if (!big.e) {
      PyErr_NoMemory();
      return -1;
    }
    for (Py_ssize_t i = 0; i < m->cap; i++)
      if (m->e[i].v) *memo_slot(&big, m->e[i].w) = m->e[i];
    PyMem_Free(m->e);
    m->e = big.e;
    m->cap = big.cap;
  }
  MemoEnt* e = memo_slot(m, w);
  if (!e->v) m->n++;
  memcpy(e->w, w, sizeof e->w);
  Py_INCREF(v);
  Py_XSETREF(e->v, v);
  return 0;
}

static int g_memo_check = 0;  /* memo_check(1): every memo hit is derived again and compared */
static long long g_memo_hits = 0;

static PyObject* memo_check(PyObject* self, PyObject* args) {
  int on;
  (void)self;
  if (!PyArg_ParseTuple(args, "p", &on)) return NULL;
  g_memo_check = on;
  const long long h = g_memo_hits;
  g_memo_hits = 0;
  return PyLong_FromLongLong(h);
}

/* note()'s count changes, gathered per key OBJECT in C and added to the diff dict once per
 * object at the merge's end, in first-note order -- the dict then gains its keys in the order
 * the per-call updates gave (a string's first object is noted when the string first is) and
 * the same sums, without a dict update and an int allocation per call (~5 per occurrence).
 * Each object is held while noted, so its address is not reused by another key. */
typedef struct {
  PyObject* k;
  long d;
} NoteEnt;
typedef struct {
  NoteEnt* t;        /* open addressing on the object address */
  Py_ssize_t* order; /* slots in first-note order */
  Py_ssize_t cap, n;
} Notes;

static Py_ssize_t notes_slot(const Notes* s, PyObject* k) {
  size_t h = ((size_t)(uintptr_t)k >> 4) * 0x9E3779B97F4A7C15ull;
  for (size_t i = h & (size_t)(s->cap - 1);; i = (i + 1) & (size_t)(s->cap - 1))
    if (s->t[i].k == k || !s->t[i].k) return (Py_ssize_t)i;
}

static int notes_add(Notes* s, PyObject* k, long d) {
  if (2 * (s->n + 1) > s->cap) {
    Notes g = {NULL, NULL, s->cap ? 2 * s->cap : 1024, 0};
    g.t = PyMem_Calloc(g.cap, sizeof *g.t);
    g.order = PyMem_Malloc(g.cap * sizeof *g.order);
    if (!g.t || !g.order) {
      PyMem_Free(g.t);
      PyMem_Free(g.order);
      PyErr_NoMemory();
      return -1;
    }
    for (Py_ssize_t i = 0; i < s->n; i++) {
      const NoteEnt e = s->t[s->order[i]];
      const Py_ssize_t j = notes_slot(&g, e.k);
      g.t[j] = e;
      g.order[g.n++] = j;
    }
    PyMem_Free(s->t);
    PyMem_Free(s->order);
    *s = g;
  }
  const Py_ssize_t i = notes_slot(s, k);
  if (!s->t[i].k) {
    Py_INCREF(k);
    s->t[i].k = k;
    s->t[i].d = 0;
    s->order[s->n++] = i;
  }
  s->t[i].d += d;
  return 0;
}

/* diff[k] = diff.get(k, 0) + d for every noted object in first-note order, then release them;
 * with diff NULL only release (an error path) */
static int notes_flush(Notes* s, PyObject* diff) {
  int rc = 0;
  for (Py_ssize_t i = 0; i < s->n; i++) {
    NoteEnt* e = &s->t[s->order[i]];
    if (diff && rc == 0) {
      PyObject* old = PyDict_GetItemWithError(diff, e->k);
      if (!old && PyErr_Occurred()) {
        rc = -1;
      } else {
        const long v = (old ? PyLong_AsLong(old) : 0) + e->d;
        PyObject* nv = (v == -1 && PyErr_Occurred()) ? NULL : PyLong_FromLong(v);
        rc = nv ? PyDict_SetItem(diff, e->k, nv) : -1;
        Py_XDECREF(nv);
      }
    }
    Py_DECREF(e->k);
  }
  PyMem_Free(s->t);
  PyMem_Free(s->order);
  s->t = NULL;
  s->order = NULL;
  s->cap = s->n = 0;
  return rc;
}

typedef struct {
  PyObject *chains, *gd, *pk, *edges, *edges_fn, *names, *diff;
  Memo* memo; /* the pair-key memo, or NULL (see mpair_key) */
  Notes notes;
} MSt;

static int key_error(PyObject* k) {
  PyObject* a = PyTuple_Pack(1, k);
  if (a) {
    PyErr_SetObject(PyExc_KeyError, a);
    Py_DECREF(a);
  }
  return -1;
}

static int note(MSt* m, PyObject* k, long d) { return notes_add(&m->notes, k, d); }

/* small non-negative ints (chain and bond indices) from a cache: PyLong_FromSsize_t allocates
 * every value above 256, twice or more per key and per occurrence here */
static PyObject* g_ints[1 << 16];
static PyObject* cint(Py_ssize_t v) {
  if (v >= 0 && v < (Py_ssize_t)(sizeof g_ints / sizeof g_ints[0])) {
    if (!g_ints[v] && !(g_ints[v] = PyLong_FromSsize_t(v))) return NULL;
    Py_INCREF(g_ints[v]);
    return g_ints[v];
  }
  return PyLong_FromSsize_t(v);
}

static PyObject* pair2(Py_ssize_t ci, Py_ssize_t i) {
  PyObject *a = cint(ci), *b = cint(i);
  PyObject* t = (a && b) ? PyTuple_Pack(2, a, b) : NULL;
  Py_XDECREF(a);
  Py_XDECREF(b);
  return t;
}

/* the stored key of the pair starting at bond i of the chain (pk row: the chain's list;
 * None = no pair), borrowed; NULL without an error when there is none */
static PyObject* pk_get(PyObject* row, Py_ssize_t i) {
  if (i < 0 || i >= PyList_GET_SIZE(row)) return NULL;
  PyObject* k = PyList_GET_ITEM(row, i);
  return k == Py_None ? NULL : k;
}
static int pk_set(PyObject* row, Py_ssize_t i, PyObject* k) {
  if (i < 0 || i >= PyList_GET_SIZE(row)) {
    PyErr_SetString(PyExc_IndexError, "rmsdkey.merge: pair position outside the chain");
    return -1;
  }
  PyObject* v = k ? k : Py_None;
  Py_INCREF(v);
  return PyList_SetItem(row, i, v);
}

/* the chain's column lists in json key order (a new tuple) */
static PyObject* chain_cols(MSt* m, PyObject* chain) {
  PyObject* cur = PyObject_GetAttr(chain, ATTR[A_CUR]);
  if (!cur) return NULL;
  PyObject* t = PyTuple_New(9);
  for (int i = 0; t && i < 9; i++) {
    PyObject* col = PyObject_GetItem(cur, PyTuple_GET_ITEM(m->names, i));
    if (!col) {
      Py_CLEAR(t);
      break;
    }
    PyTuple_SET_ITEM(t, i, col);
  }
  Py_DECREF(cur);
  return t;
}

static Py_ssize_t list_int(PyObject* lst, Py_ssize_t i) {
  if (i < 0 || i >= PyList_GET_SIZE(lst)) {
    PyErr_SetString(PyExc_IndexError, "list index out of range");
    return -1;
  }
  return PyLong_AsSsize_t(PyList_GET_ITEM(lst, i));
}

/* RmsdBPE._pair_key(c, i1, la, lb) (bpe.py:1192-1299) */
static PyObject* mpair_key(MSt* m, PyObject* cols, PyObject* init, PyObject* tp, PyObject* btt, Py_ssize_t nres,
                           Py_ssize_t i1, Py_ssize_t la, Py_ssize_t lb) {
  const Py_ssize_t p1 = list_int(tp, i1), p2 = p1 < 0 ? -1 : list_int(tp, i1 + la);
  if (p1 < 0 || p2 < 0) return NULL;
  PyObject *k1 = cint(p1), *k2 = cint(p2);
  PyObject* t1 = k1 ? PyDict_GetItemWithError(btt, k1) : NULL;
  PyObject* t2 = (t1 && k2) ? PyDict_GetItemWithError(btt, k2) : NULL;
  if (!t1 || !t2) {
    if (!PyErr_Occurred()) key_error(!t1 ? k1 : k2);
    Py_XDECREF(k1);
    Py_XDECREF(k2);
    return NULL;
  }
  Py_DECREF(k1);
  Py_DECREF(k2);
  const int same = PyObject_RichCompareBool(PyTuple_GET_ITEM(t1, 0), PyTuple_GET_ITEM(t2, 0), Py_EQ);
  if (same < 0) return NULL;
  if (same) {
    PyErr_SetString(PyExc_RuntimeError, "pair of one token");
    return NULL;
  }
  const int pt1 = PyTuple_Check(PyTuple_GET_ITEM(t1, 1)), pt2 = PyTuple_Check(PyTuple_GET_ITEM(t2, 1));
  const Py_ssize_t L = la + lb;
  Py_ssize_t lo[3], hi[3];
  if (pt1 && pt2) {
    lo[0] = 0, hi[0] = 0, lo[1] = la - 1, hi[1] = la, lo[2] = la - 2, hi[2] = la;
  } else if (pt1) {
    lo[0] = la, hi[0] = L, lo[1] = la - 1, hi[1] = L, lo[2] = la - 2, hi[2] = L;
  } else if (pt2) {
    lo[0] = 0, hi[0] = la, lo[1] = 0, hi[1] = la, lo[2] = 0, hi[2] = la;
  } else {
    lo[0] = 0, hi[0] = L, lo[1] = 0, hi[1] = L, lo[2] = 0, hi[2] = L;
  }
  if (i1 + L - 1 > 3 * nres - 1) {
    PyErr_Format(PyExc_ValueError, "idx+l cannot exceed %zd", 3 * nres - 1);
    return NULL;
  }
  /* Memo (m->memo, the RMSD mode without glue optimisation): a pair of two partitioned tokens
   * keys on raw values everywhere but the junction -- the angle at span position la - 1 and
   * the dihedrals at la - 2, la - 1 (lo / hi above) -- and each token's raw values are its
   * medoid geometry, written whole by set_token_geo when the token was made (bpe.py:1974-1985,
   * 294-330) and never touched again.  So the key string is a function of (token ids, span
   * length, phase, the three junction values): a merge's occurrences share most of them. */
  int use_memo = 0;
  long long w[9];
  if (m->memo && pt1 && pt2 && la >= 2 && i1 + la - 2 >= 0) {
    static const int BA[3] = {8, 3, 1}, DH[3] = {7, 5, 6};
    PyObject *id1 = PyTuple_GET_ITEM(t1, 1), *id2 = PyTuple_GET_ITEM(t2, 1);
    int ok = PyTuple_GET_SIZE(id1) == 2 && PyTuple_GET_SIZE(id2) == 2;
    for (int q = 0; ok && q < 2; q++) {
      w[q] = PyLong_AsLongLong(PyTuple_GET_ITEM(id1, q));
      w[2 + q] = PyLong_AsLongLong(PyTuple_GET_ITEM(id2, q));
    }
    if (PyErr_Occurred()) return NULL;
    w[4] = (long long)L;
    w[5] = (long long)(i1 % 3);
    const Py_ssize_t a = i1 + la - 1, d0 = i1 + la - 2;
    double v[3];
    for (int q = 0; ok && q < 3; q++) {
      PyObject* col;
      Py_ssize_t row;
      if (q == 0) {
        if (a == 0) { /* (the init angle) */
          v[0] = PyFloat_AsDouble(PyList_GET_ITEM(init, 2));
          continue;
        }
        col = PyTuple_GET_ITEM(cols, BA[a % 3]);
        row = (a - 1) / 3;
      } else {
        const Py_ssize_t d = d0 + (q - 1);
        col = PyTuple_GET_ITEM(cols, DH[d % 3]);
        row = (d + 1) / 3;
      }
      if (row < 0 || row >= PyList_GET_SIZE(col)) {
        ok = 0;
        break;
      }
      v[q] = PyFloat_AsDouble(PyList_GET_ITEM(col, row));
    }
    if (PyErr_Occurred()) return NULL;
    if (ok) {
      memcpy(&w[6], v, sizeof v);
      use_memo = 1;
      PyObject* hit = memo_slot(m->memo, w)->v;
      if (hit && !g_memo_check) {
        Py_INCREF(hit);
        return hit;
      }
      if (hit) g_memo_hits++;  /* (check mode: derived below and compared) */
    }
  }
  PyObject* kL = cint(L);
  if (!kL) return NULL;
  PyObject* thr = PyDict_GetItemWithError(m->edges, kL);
  if (thr) {
    Py_INCREF(thr);
  } else if (!PyErr_Occurred()) {
    thr = PyObject_CallOneArg(m->edges_fn, kL);  /* (computes and caches it) */
  }
  Py_DECREF(kL);
  if (!thr) return NULL;
  if (!PyTuple_Check(thr) || PyTuple_GET_SIZE(thr) != 9) {
    Py_DECREF(thr);
    PyErr_SetString(PyExc_TypeError, "rmsdkey.merge: edges must be a 9-tuple");
    return NULL;
  }
  PROF_T(pk0);
  PyObject* k = build_key(cols, init, i1, L, i1 % 3, lo, hi, thr);
  PROF_ADD(6, pk0);
  Py_DECREF(thr);
  if (use_memo && k) {
    PyObject* hit = memo_slot(m->memo, w)->v;
    if (hit) { /* (check mode) */
      if (PyUnicode_Compare(hit, k) != 0) {
        PyErr_Format(PyExc_AssertionError, "rmsdkey: memo key %R differs from the derived key %R", hit, k);
        Py_CLEAR(k);
      }
    } else if (memo_put(m->memo, w, k) < 0) {
      Py_CLEAR(k);
    }
  }
  return k;
}

static int set_in(MSt* m, PyObject* k, PyObject* item, int add) {
  PyObject* set = PyObject_GetItem(m->gd, k);  /* (defaultdict: a missing key gets a new set) */
  if (!set) return -1;
  int rc;
  if (add) {
    rc = PySet_Add(set, item);
  } else {
    rc = PySet_Discard(set, item);
    if (rc == 0) rc = key_error(item);
    else if (rc == 1) rc = 0;
  }
  Py_DECREF(set);
  return rc;
}

static int apply_geo(PyObject* chain, PyObject* cols, PyObject* init, Py_ssize_t i1, Py_ssize_t len, PyObject* vals) {
  int rc = PyDict_CheckExact(vals) ? setgeo_impl(cols, init, i1, len, vals) : 0;
  if (rc != 0) return rc < 0 ? -1 : 0;
  PyObject* r = PyObject_CallMethod(chain, "set_geo", "nnO", i1, len, vals);  /* (the Python path: its errors) */
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

static PyObject* merge(PyObject* self, PyObject* args) {
  PyObject *st, *occs, *assigns, *key, *vals, *diff;
  Py_ssize_t length, n;
  int rmsd;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!OUnnpOO!", &PyTuple_Type, &st, &PyList_Type, &occs, &assigns, &key, &length, &n,
                        &rmsd, &vals, &PyDict_Type, &diff))
    return NULL;
  MSt m;
  PyObject* memo = NULL;
  if (!PyArg_ParseTuple(st, "O!OO!O!OO!|O", &PyList_Type, &m.chains, &m.gd, &PyList_Type, &m.pk, &PyDict_Type, &m.edges,
                        &m.edges_fn, &PyTuple_Type, &m.names, &memo))
    return NULL;
  m.memo = NULL;
  if (memo && memo != Py_None) {
    m.memo = (Memo*)PyCapsule_GetPointer(memo, MEMO_NAME);
    if (!m.memo) return NULL;
  }
  m.diff = diff;
  m.notes = (Notes){NULL, NULL, 0, 0};
  PyObject* nobj = PyLong_FromSsize_t(n);
  PyObject* lenobj = PyLong_FromSsize_t(length);
  PyObject *chain = NULL, *cols = NULL, *init = NULL, *tp = NULL, *btt = NULL, *events = NULL, *nres_o = NULL;
  PyObject *t12 = NULL, *t01 = NULL, *t23 = NULL, *left = NULL, *right = NULL, *pkrow = NULL;
  Py_ssize_t cur_ci = -1, nres = 0, last_ci = -1, last_i1 = 0;
  int have_last = 0, err = 0;
  /* the merged key's set, looked up once (every removal below is from it); NULL: per call */
  PyObject* kset = PyDict_Check(m.gd) ? PyDict_GetItemWithError(m.gd, key) : NULL;
  if (!kset && PyErr_Occurred()) goto fail;
  if (kset && !PySet_Check(kset)) kset = NULL;
  Py_XINCREF(kset);
  if (!nobj || !lenobj) goto fail;
  for (Py_ssize_t q = 0; q < PyList_GET_SIZE(occs); q++) {
    PyObject* oc = PyList_GET_ITEM(occs, q);  /* (the very tuples _geo_dict's sets hold) */
    if (!PyTuple_CheckExact(oc) || PyTuple_GET_SIZE(oc) != 2) {
      PyErr_SetString(PyExc_TypeError, "rmsdkey.merge: occurrences must be (chain, index) tuples");
      goto fail;
    }
    const Py_ssize_t ci = PyLong_AsSsize_t(PyTuple_GET_ITEM(oc, 0)), i2 = PyLong_AsSsize_t(PyTuple_GET_ITEM(oc, 1));
    if ((ci == -1 || i2 == -1) && PyErr_Occurred()) goto fail;
    if (ci != cur_ci) {  /* the chain's objects, kept while its occurrences run */
      Py_CLEAR(cols);
      Py_CLEAR(init);
      Py_CLEAR(tp);
      Py_CLEAR(btt);
      Py_CLEAR(events);
      Py_CLEAR(nres_o);
      if (ci < 0 || ci >= PyList_GET_SIZE(m.chains)) {
        PyErr_SetString(PyExc_IndexError, "chain index out of range");
        goto fail;
      }
      chain = PyList_GET_ITEM(m.chains, ci);
      cols = chain_cols(&m, chain);
      init = PyObject_GetAttr(chain, ATTR[A_INIT]);
      tp = PyObject_GetAttr(chain, ATTR[A_TOKEN_POS]);
      btt = PyObject_GetAttr(chain, ATTR[A_BTT]);
      events = PyObject_GetAttr(chain, ATTR[A_EVENTS]);
      nres_o = PyObject_GetAttr(chain, ATTR[A_N]);
      if (!cols || !init || !tp || !btt || !events || !nres_o) goto fail;
      if (!PyList_Check(tp) || !PyDict_Check(btt) || !PyList_Check(events) || !PyList_Check(init)) {
        PyErr_SetString(PyExc_TypeError, "rmsdkey.merge: unexpected chain state");
        goto fail;
      }
      nres = PyLong_AsSsize_t(nres_o);
      if (ci >= PyList_GET_SIZE(m.pk) || !PyList_Check(PyList_GET_ITEM(m.pk, ci))) {
        PyErr_SetString(PyExc_TypeError, "rmsdkey.merge: the pair keys must be one list per chain");
        goto fail;
      }
      pkrow = PyList_GET_ITEM(m.pk, ci);  /* (borrowed: m.pk holds it) */
      cur_ci = ci;
    }
    PROF_T(pt0);
    const Py_ssize_t i1 = list_int(tp, i2 - 1);
    if (i1 < 0 && PyErr_Occurred()) goto fail;
    const Py_ssize_t l1 = i2 - i1, l2 = length - l1;
    if (have_last && last_ci == ci && last_i1 + length > i1) continue;  /* overlaps (bpe.py:1909-1912) */
    if (!(l1 > 0 && l2 > 0)) {
      PyErr_SetString(PyExc_AssertionError, "bad split");
      goto fail;
    }
    t12 = oc;
    Py_INCREF(t12);
    PyObject* cur_key = pk_get(pkrow, i2);
    const int same = cur_key ? PyObject_RichCompareBool(cur_key, key, Py_EQ) : 0;
    if (same < 0) goto fail;
    if (!same) {  /* bpe.py:1917-1920 */
      Py_CLEAR(t12);
      continue;
    }
    if (kset) {
      const int rc = PySet_Discard(kset, t12);
      if (rc < 0 || (rc == 0 && key_error(t12) < 0)) goto fail;
    } else if (set_in(&m, key, t12, 0) < 0) {
      goto fail;
    }
    if (pk_set(pkrow, i2, NULL) < 0 || note(&m, key, -1) < 0) goto fail;
    Py_ssize_t i0 = 0, l0 = 0, i3 = 0, l3 = 0;
    const Py_ssize_t ntp = PyList_GET_SIZE(tp);
    if (i1) {
      i0 = list_int(tp, i1 - 1);
      if (i0 < 0 && PyErr_Occurred()) goto fail;
      l0 = i1 - i0;
      t01 = pair2(ci, i1);
      if (!t01) goto fail;
      left = pk_get(pkrow, i1);
      if (!left) {
        key_error(t01);
        goto fail;
      }
      Py_INCREF(left);
    }
    if (i2 + l2 < ntp) {
      i3 = i2 + l2;
      l3 = 0;
      while (i3 + l3 < ntp) {
        const Py_ssize_t v = list_int(tp, i3 + l3);
        if (v < 0 && PyErr_Occurred()) goto fail;
        if (v != i3) break;
        l3++;
      }
      t23 = pair2(ci, i3);
      if (!t23) goto fail;
      right = pk_get(pkrow, i3);
      if (!right) {
        key_error(t23);
        goto fail;
      }
      Py_INCREF(right);
    }
    if (left && (set_in(&m, left, t01, 0) < 0 || note(&m, left, -1) < 0)) goto fail;
    if (right && (set_in(&m, right, t23, 0) < 0 || note(&m, right, -1) < 0)) goto fail;
    PROF_ADD(0, pt0);
    {
      PyObject* vi1 = cint(i1);
      if (!vi1) goto fail;
      for (Py_ssize_t j = i2; j < i2 + l2; j++) {
        Py_INCREF(vi1);
        if (PyList_SetItem(tp, j, vi1) < 0) {
          Py_DECREF(vi1);
          goto fail;
        }
      }
      PyObject* ki2 = cint(i2);
      int rc = ki2 ? PyDict_DelItem(btt, ki2) : -1;
      Py_XDECREF(ki2);
      PyObject *tokid = NULL, *val = NULL, *ev = NULL;
      if (rc == 0) {
        if (rmsd) {
          PyObject* a = PyList_GET_ITEM(assigns, q);
          tokid = PyTuple_Pack(2, nobj, a);
        } else {
          tokid = nobj;
          Py_INCREF(tokid);
        }
        val = tokid ? PyTuple_Pack(3, vi1, tokid, lenobj) : NULL;
        rc = val ? PyDict_SetItem(btt, vi1, val) : -1;
        if (rc == 0) {
          PyObject* vi2 = cint(i2);
          ev = vi2 ? PyTuple_Pack(3, vi1, vi2, val) : NULL;
          Py_XDECREF(vi2);
          rc = ev ? PyList_Append(events, ev) : -1;
        }
      }
      Py_XDECREF(tokid);
      Py_XDECREF(val);
      Py_XDECREF(ev);
      Py_DECREF(vi1);
      if (rc < 0) goto fail;
    }
    PROF_ADD(1, pt0);
    if (rmsd && vals != Py_None) {  /* (None: rmsd_only, the merge keeps its own geometry) */
      PyObject* a = PyList_GET_ITEM(assigns, q);
      PyObject* struc = PyObject_GetItem(vals, a);
      if (!struc) goto fail;
      const int rc = apply_geo(chain, cols, init, i1, length, struc);
      Py_DECREF(struc);
      if (rc < 0) goto fail;
    }
    PROF_ADD(2, pt0);
    if (left) {
      PyObject* k = mpair_key(&m, cols, init, tp, btt, nres, i0, l0, length);
      PROF_ADD(3, pt0);
      if (!k) goto fail;
      const int rc = (set_in(&m, k, t01, 1) < 0 || pk_set(pkrow, i1, k) < 0 || note(&m, k, 1) < 0) ? -1 : 0;
      Py_DECREF(k);
      PROF_ADD(4, pt0);
      if (rc < 0) goto fail;
    }
    if (right) {
      PyObject* k = mpair_key(&m, cols, init, tp, btt, nres, i1, length, l3);
      PROF_ADD(3, pt0);
      if (!k) goto fail;
      const int rc = (set_in(&m, k, t23, 1) < 0 || pk_set(pkrow, i3, k) < 0 || note(&m, k, 1) < 0) ? -1 : 0;
      Py_DECREF(k);
      PROF_ADD(4, pt0);
      if (rc < 0) goto fail;
    }
    if (!rmsd && apply_geo(chain, cols, init, i1, length, vals) < 0) goto fail;
    PROF_ADD(5, pt0);
    last_ci = ci;
    last_i1 = i1;
    have_last = 1;
    Py_CLEAR(t12);
    Py_CLEAR(t01);
    Py_CLEAR(t23);
    Py_CLEAR(left);
    Py_CLEAR(right);
  }
  goto done;
fail:
  err = 1;
done:
  if (notes_flush(&m.notes, err ? NULL : diff) < 0) err = 1;
  Py_XDECREF(kset);
  Py_XDECREF(t12);
  Py_XDECREF(t01);
  Py_XDECREF(t23);
  Py_XDECREF(left);
  Py_XDECREF(right);
  Py_XDECREF(cols);
  Py_XDECREF(init);
  Py_XDECREF(tp);
  Py_XDECREF(btt);
  Py_XDECREF(events);
  Py_XDECREF(nres_o);
  Py_XDECREF(nobj);
  Py_XDECREF(lenobj);
  if (err) return NULL;
  Py_RETURN_NONE;
}

/* rekey(st, cis, diff) -- the re-keying after a merge's glue re-optimisation (RmsdBPE._merge,
 * bpe.py:2027-2071): for every chain ci of cis, every token of its btt (insertion order) but the
 * chain's last, the key of the pair it starts is derived afresh from the re-optimised glues; a
 * changed key moves the pair between the sets: gd[old].remove((ci, i2)), gd[new].add((ci, i2)),
 * pk[ci][i2] = new, diff[old] - 1, diff[new] + 1.  st as merge's (its memo unused: the glues inside
 * the tokens changed).  The Python loop it replaces ran ~45 dict / set / tuple operations a pair
 * over every pair of every touched chain: ~3/4 of the README setting's host time a step. */
static PyObject* rekey(PyObject* self, PyObject* args) {
  PyObject *st, *cis, *diff;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!O!", &PyTuple_Type, &st, &PyList_Type, &cis, &PyDict_Type, &diff)) return NULL;
  MSt m;
  PyObject* memo = NULL;
  if (!PyArg_ParseTuple(st, "O!OO!O!OO!|O", &PyList_Type, &m.chains, &m.gd, &PyList_Type, &m.pk, &PyDict_Type, &m.edges,
                        &m.edges_fn, &PyTuple_Type, &m.names, &memo))
    return NULL;
  m.memo = NULL;
  m.diff = diff;
  m.notes = (Notes){NULL, NULL, 0, 0};
  int err = 0;
  for (Py_ssize_t q = 0; q < PyList_GET_SIZE(cis) && !err; q++) {
    const Py_ssize_t ci = PyLong_AsSsize_t(PyList_GET_ITEM(cis, q));
    if (ci == -1 && PyErr_Occurred()) {
      err = 1;
      break;
    }
    if (ci < 0 || ci >= PyList_GET_SIZE(m.chains) || ci >= PyList_GET_SIZE(m.pk)) {
      PyErr_SetString(PyExc_IndexError, "chain index out of range");
      err = 1;
      break;
    }
    PyObject* chain = PyList_GET_ITEM(m.chains, ci);
    PyObject* pkrow = PyList_GET_ITEM(m.pk, ci);
    PyObject* cols = chain_cols(&m, chain);
    PyObject* init = PyObject_GetAttr(chain, ATTR[A_INIT]);
    PyObject* tp = PyObject_GetAttr(chain, ATTR[A_TOKEN_POS]);
    PyObject* btt = PyObject_GetAttr(chain, ATTR[A_BTT]);
    PyObject* nres_o = PyObject_GetAttr(chain, ATTR[A_N]);
    PyObject* items = NULL;
    if (!cols || !init || !tp || !btt || !nres_o || !PyList_Check(pkrow)) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "rmsdkey.rekey: unexpected chain state");
      err = 1;
    } else if (!PyList_Check(tp) || !PyDict_Check(btt) || !PyList_Check(init)) {
      PyErr_SetString(PyExc_TypeError, "rmsdkey.rekey: unexpected chain state");
      err = 1;
    } else {
      items = PyDict_Items(btt);  /* (a snapshot, as list(btt.items())) */
      if (!items) err = 1;
    }
    const Py_ssize_t nres = err ? 0 : PyLong_AsSsize_t(nres_o);
    if (!err && nres == -1 && PyErr_Occurred()) err = 1;
    const Py_ssize_t last = 3 * nres - 1;
    for (Py_ssize_t e = 0; !err && e < PyList_GET_SIZE(items); e++) {
      PyObject* it = PyList_GET_ITEM(items, e);
      PyObject* v = PyTuple_GET_ITEM(it, 1);
      const Py_ssize_t i1 = PyLong_AsSsize_t(PyTuple_GET_ITEM(it, 0));
      const Py_ssize_t l1 = PyTuple_Check(v) && PyTuple_GET_SIZE(v) == 3 ? PyLong_AsSsize_t(PyTuple_GET_ITEM(v, 2)) : -1;
      if (PyErr_Occurred() || l1 < 0) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "rmsdkey.rekey: btt entries must be 3-tuples");
        err = 1;
        break;
      }
      if (i1 + l1 == last) continue;
      const Py_ssize_t i2 = i1 + l1;
      PyObject* k2 = cint(i2);
      PyObject* v2 = k2 ? PyDict_GetItemWithError(btt, k2) : NULL;
      if (!v2) {
        if (k2 && !PyErr_Occurred()) key_error(k2);
        Py_XDECREF(k2);
        err = 1;
        break;
      }
      Py_DECREF(k2);
      const Py_ssize_t l2 = PyLong_AsSsize_t(PyTuple_GET_ITEM(v2, 2));
      if (l2 == -1 && PyErr_Occurred()) {
        err = 1;
        break;
      }
      PyObject* old = pk_get(pkrow, i2);
      PyObject* t = pair2(ci, i2);
      if (!t) {
        err = 1;
        break;
      }
      if (!old) {  /* (_pk_at: KeyError((ci, i2))) */
        key_error(t);
        Py_DECREF(t);
        err = 1;
        break;
      }
      Py_INCREF(old);
      PyObject* nk = mpair_key(&m, cols, init, tp, btt, nres, i1, l1, l2);
      const int same = nk ? PyObject_RichCompareBool(nk, old, Py_EQ) : -1;
      if (same < 0) {
        err = 1;
      } else if (!same) {
        if (set_in(&m, old, t, 0) < 0 || note(&m, old, -1) < 0 || set_in(&m, nk, t, 1) < 0 || pk_set(pkrow, i2, nk) < 0 ||
            note(&m, nk, 1) < 0)
          err = 1;
      }
      Py_XDECREF(nk);
      Py_DECREF(old);
      Py_DECREF(t);
    }
    Py_XDECREF(items);
    Py_XDECREF(cols);
    Py_XDECREF(init);
    Py_XDECREF(tp);
    Py_XDECREF(btt);
    Py_XDECREF(nres_o);
  }
  if (notes_flush(&m.notes, err ? NULL : diff) < 0) err = 1;
  if (err) return NULL;
  Py_RETURN_NONE;
}

/* prio(diff, k2p, heap, push, gd, spheres) -- step 7 of BPE.step (bpe.py:2077-2138) as
 * RmsdBPE._merge runs it: every key whose count changed leaves the priority queue and comes
 * back with its new count (flag = not partitioned, -count, key); a key whose count reached 0
 * leaves _geo_dict.  The queue is rmsd_bpe._PrioQueue: k2p is its live map (dropping a key's
 * entry from k2p removes it), heap / push its heap list and heapq.heappush. */
static PyObject* prio(PyObject* self, PyObject* args) {
  PyObject *diff, *k2p, *heap, *push, *gd, *spheres;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!O!OOO", &PyDict_Type, &diff, &PyDict_Type, &k2p, &PyList_Type, &heap, &push, &gd,
                        &spheres))
    return NULL;
  Py_ssize_t it = 0;
  PyObject *k, *d;
  while (PyDict_Next(diff, &it, &k, &d)) {
    long count = 0;
    PyObject* pr = PyDict_GetItemWithError(k2p, k);
    if (!pr && PyErr_Occurred()) return NULL;
    if (pr) {
      count = -PyLong_AsLong(PyTuple_GET_ITEM(pr, 1));
      if (PyDict_DelItem(k2p, k) < 0) return NULL;  /* (pr is gone with it) */
    }
    count += PyLong_AsLong(d);
    if (PyErr_Occurred()) return NULL;
    PyObject* set = PyObject_GetItem(gd, k);  /* (defaultdict: as len(gd[k])) */
    if (!set) return NULL;
    const Py_ssize_t n = PySet_Size(set);
    Py_DECREF(set);
    if (n < 0) return NULL;
    if (count != n) {
      PyObject* head = PyUnicode_Substring(k, 0, 60);
      if (head) {
        PyErr_Format(PyExc_AssertionError, "count of %U out of step", head);
        Py_DECREF(head);
      }
      return NULL;
    }
    if (count) {
      const int in = PySequence_Contains(spheres, k);
      if (in < 0) return NULL;
      PyObject* negc = PyLong_FromLong(-count);
      PyObject* npr = negc ? PyTuple_Pack(3, in ? Py_False : Py_True, negc, k) : NULL;
      Py_XDECREF(negc);
      if (!npr) return NULL;
      if (PyDict_SetItem(k2p, k, npr) < 0) {
        Py_DECREF(npr);
        return NULL;
      }
      PyObject* r = PyObject_CallFunctionObjArgs(push, heap, npr, NULL);
      Py_DECREF(npr);
      if (!r) return NULL;
      Py_DECREF(r);
    } else if (PyDict_DelItem(gd, k) < 0) {
      return NULL;
    }
  }
  Py_RETURN_NONE;
}

/* packc(chains, orig, spans, out) -- pack() with the spans given as (chain index, q, r): the
 * chain's columns (cur, or orig) and init are read here (PACK order below) */
static const char* PACK_NAMES[9] = {"N:CA", "CA:C", "tau", "0C:1N", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"};
static PyObject* packc(PyObject* self, PyObject* args) {
  PyObject *chains, *spans;
  Py_buffer out;
  int orig;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!pO!w*", &PyList_Type, &chains, &orig, &PyList_Type, &spans, &out)) return NULL;
  double* o = (double*)out.buf;
  const Py_ssize_t cap = out.len / (Py_ssize_t)sizeof(double);
  Py_ssize_t at = 0, last_ci = -1;
  PyObject* cols = NULL;
  PyObject* init = NULL;
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(spans); i++) {
    Py_ssize_t ci, q, r;
    if (!PyArg_ParseTuple(PyList_GET_ITEM(spans, i), "nnn", &ci, &q, &r)) goto fail;
    if (ci != last_ci) {
      Py_CLEAR(cols);
      Py_CLEAR(init);
      if (ci < 0 || ci >= PyList_GET_SIZE(chains)) {
        PyErr_SetString(PyExc_IndexError, "chain index out of range");
        goto fail;
      }
      PyObject* c = PyList_GET_ITEM(chains, ci);
      PyObject* src = PyObject_GetAttr(c, ATTR[orig ? A_ORIG : A_CUR]);
      init = PyObject_GetAttr(c, ATTR[A_INIT]);
      if (!src || !init) {
        Py_XDECREF(src);
        goto fail;
      }
      cols = PyTuple_New(9);
      for (int t = 0; cols && t < 9; t++) {
        PyObject* col = PyObject_GetItem(src, PACK_KEYS[t]);
        if (!col) {
          Py_CLEAR(cols);
          break;
        }
        PyTuple_SET_ITEM(cols, t, col);
      }
      Py_DECREF(src);
      if (!cols) goto fail;
      if (!PyList_Check(init) || PyList_GET_SIZE(init) < 3) {
        PyErr_SetString(PyExc_TypeError, "rmsdkey.packc: init must be a list of 3");
        goto fail;
      }
      for (int t = 0; t < 9; t++)
        if (!PyList_Check(PyTuple_GET_ITEM(cols, t))) {
          PyErr_SetString(PyExc_TypeError, "rmsdkey.packc: columns must be lists");
          goto fail;
        }
      last_ci = ci;
    }
    if (q < 0 || r < 1 || at + 9 * r > cap) {
      PyErr_SetString(PyExc_ValueError, "rmsdkey.packc: bad span");
      goto fail;
    }
    if (pack_one(cols, init, q, r, o + at) < 0) goto fail;
    at += 9 * r;
  }
  Py_CLEAR(cols);
  Py_CLEAR(init);
  PyBuffer_Release(&out);
  return PyLong_FromSsize_t(at / 9);
fail:
  Py_XDECREF(cols);
  Py_XDECREF(init);
  PyBuffer_Release(&out);
  return NULL;
}

/* packa(chains, orig, spans, out) -- packc() with the spans an int64 (n, 3) buffer of
 * (chain index, q, r) rows (no tuple per span) */
static PyObject* packa(PyObject* self, PyObject* args) {
  PyObject* chains;
  Py_buffer sb, out;
  int orig;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!py*w*", &PyList_Type, &chains, &orig, &sb, &out)) return NULL;
  double* o = (double*)out.buf;
  const Py_ssize_t cap = out.len / (Py_ssize_t)sizeof(double);
  const int64_t* sp = (const int64_t*)sb.buf;
  const Py_ssize_t ns = sb.len / (3 * (Py_ssize_t)sizeof(int64_t));
  Py_ssize_t at = 0, last_ci = -1;
  PyObject* cols = NULL;
  PyObject* init = NULL;
  int err = 0;
  for (Py_ssize_t i = 0; i < ns && !err; i++) {
    const Py_ssize_t ci = (Py_ssize_t)sp[3 * i], q = (Py_ssize_t)sp[3 * i + 1], r = (Py_ssize_t)sp[3 * i + 2];
    if (ci != last_ci) {
      Py_CLEAR(cols);
      Py_CLEAR(init);
      if (ci < 0 || ci >= PyList_GET_SIZE(chains)) {
        PyErr_SetString(PyExc_IndexError, "chain index out of range");
        err = 1;
        break;
      }
      PyObject* c = PyList_GET_ITEM(chains, ci);
      PyObject* src = PyObject_GetAttr(c, ATTR[orig ? A_ORIG : A_CUR]);
      init = PyObject_GetAttr(c, ATTR[A_INIT]);
      cols = (src && init) ? PyTuple_New(9) : NULL;
      for (int t = 0; cols && t < 9; t++) {
        PyObject* col = PyObject_GetItem(src, PACK_KEYS[t]);
        if (!col || !PyList_Check(col)) {
          if (col) PyErr_SetString(PyExc_TypeError, "rmsdkey.packa: columns must be lists");
          Py_XDECREF(col);
          Py_CLEAR(cols);
          break;
        }
        PyTuple_SET_ITEM(cols, t, col);
      }
      Py_XDECREF(src);
      if (!cols || !PyList_Check(init) || PyList_GET_SIZE(init) < 3) {
        if (cols) PyErr_SetString(PyExc_TypeError, "rmsdkey.packa: init must be a list of 3");
        err = 1;
        break;
      }
      last_ci = ci;
    }
    if (q < 0 || r < 1 || at + 9 * r > cap) {
      PyErr_SetString(PyExc_ValueError, "rmsdkey.packa: bad span");
      err = 1;
      break;
    }
    if (pack_one(cols, init, q, r, o + at) < 0) err = 1;
    at += 9 * r;
  }
  Py_XDECREF(cols);
  Py_XDECREF(init);
  PyBuffer_Release(&sb);
  PyBuffer_Release(&out);
  return err ? NULL : PyLong_FromSsize_t(at / 9);
}

/* spans_occ(chains, occ, length, out) -- [(ci, chains[ci].token_pos[i2 - 1], length) for ci, i2
 * in occ] (RmsdBPE._partition / the recurring merge, bpe.py:1759-1763) into an int64 (n, 3)
 * buffer */
static PyObject* spans_occ(PyObject* self, PyObject* args) {
  PyObject *chains, *occ;
  Py_ssize_t length;
  Py_buffer out;
  (void)self;
  if (!PyArg_ParseTuple(args, "O!O!nw*", &PyList_Type, &chains, &PyList_Type, &occ, &length, &out)) return NULL;
  int64_t* o = (int64_t*)out.buf;
  const Py_ssize_t n = PyList_GET_SIZE(occ);
  int err = out.len < 3 * n * (Py_ssize_t)sizeof(int64_t);
  if (err) PyErr_SetString(PyExc_ValueError, "rmsdkey.spans_occ: output too small");
  for (Py_ssize_t i = 0; i < n && !err; i++) {
    PyObject* oc = PyList_GET_ITEM(occ, i);
    if (!PyTuple_Check(oc) || PyTuple_GET_SIZE(oc) != 2) {
      PyErr_SetString(PyExc_TypeError, "rmsdkey.spans_occ: occurrences must be (chain, index) tuples");
      err = 1;
      break;
    }
    const Py_ssize_t ci = PyLong_AsSsize_t(PyTuple_GET_ITEM(oc, 0)), i2 = PyLong_AsSsize_t(PyTuple_GET_ITEM(oc, 1));
    if (PyErr_Occurred()) {
      err = 1;
      break;
    }
    if (ci < 0 || ci >= PyList_GET_SIZE(chains)) {
      PyErr_SetString(PyExc_IndexError, "chain index out of range");
      err = 1;
      break;
    }
    PyObject* tp = PyObject_GetAttr(PyList_GET_ITEM(chains, ci), ATTR[A_TOKEN_POS]);
    if (!tp || !PyList_Check(tp)) {
      if (tp) PyErr_SetString(PyExc_TypeError, "rmsdkey.spans_occ: token_pos must be a list");
      Py_XDECREF(tp);
      err = 1;
      break;
    }
    /* (Python's tp[i2 - 1]: a negative index counts from the end) */
    const Py_ssize_t j = i2 - 1 < 0 ? i2 - 1 + PyList_GET_SIZE(tp) : i2 - 1;
    const Py_ssize_t i1 = list_int(tp, j);
    Py_DECREF(tp);
    if (i1 == -1 && PyErr_Occurred()) {
      err = 1;
      break;
    }
    o[3 * i] = ci, o[3 * i + 1] = i1, o[3 * i + 2] = length;
  }
  PyBuffer_Release(&out);
  if (err) return NULL;
  Py_RETURN_NONE;
}

/* ---------------------------------------------------------------- k-medoids
 * kmed_step(D, medoids, assign) -> list -- the body of one iteration of algo.k_medoids
 * (algo.py:191-213) as rmsd.k_medoids_from_matrix runs it on the float32 (N, N) matrix D:
 * assign[i] = argmin_j D[i, medoids[j]] (np.argmin over D[:, medoids], axis 1), then per
 * cluster j the member minimising D[np.ix_(members, members)].sum(axis=1), or -1 for an
 * empty cluster (the caller draws its rng.integers(N) in j order, as there).  The row sums
 * follow numpy's float32 reduction order exactly (pairwise summation over the gathered row:
 * below 8 items a running sum, up to 128 eight accumulators, above that halves cut at a
 * multiple of 8), and argmin keeps numpy's rules (the first minimum; a NaN wins), so the
 * medoids are the numpy loop's bit for bit (tests/test_rmsd.py checks both on random and
 * tied matrices).  The numpy path gathered the members x members block per cluster (~0.7 ms
 * of a 2 000-chain RMSD step). */
static float pw_sum(const float* row, const Py_ssize_t* ix, Py_ssize_t n) {
  if (n < 8) {
    float r = 0.f;
    for (Py_ssize_t i = 0; i < n; i++) r += row[ix[i]];
    return r;
  }
  if (n <= 128) {
    float r[8];
    for (int j = 0; j < 8; j++) r[j] = row[ix[j]];
    Py_ssize_t i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; j++) r[j] += row[ix[i + j]];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += row[ix[i]];
    return res;
  }
  Py_ssize_t n2 = n / 2;
  n2 -= n2 % 8;
  const float a = pw_sum(row, ix, n2);
  return a + pw_sum(row, ix + n2, n - n2);
}

/* np.argmin's pick among v[0..n): the first NaN, else the first minimum */
static Py_ssize_t argmin_f32(const float* v, Py_ssize_t n) {
  Py_ssize_t b = 0;
  if (v[0] != v[0]) return 0;
  for (Py_ssize_t i = 1; i < n; i++) {
    if (v[i] != v[i]) return i;
    if (v[i] < v[b]) b = i;
  }
  return b;
}

static PyObject* kmed_step(PyObject* self, PyObject* args) {
  Py_buffer Db, Ab;
  PyObject* med;
  (void)self;
  if (!PyArg_ParseTuple(args, "y*O!w*", &Db, &PyList_Type, &med, &Ab)) return NULL;
  PyObject* out = NULL;
  Py_ssize_t *mi = NULL, *cnt = NULL, *mem = NULL, *start = NULL;
  float *vals = NULL, *intra = NULL;
  const Py_ssize_t k = PyList_GET_SIZE(med);
  const Py_ssize_t N = Ab.len / (Py_ssize_t)sizeof(int64_t);
  if (Db.len != N * N * (Py_ssize_t)sizeof(float) || k < 1 || N < 1) {
    PyErr_SetString(PyExc_ValueError, "rmsdkey.kmed_step: D must be float32 (N, N) and assign int64 (N,)");
    goto done;
  }
  const float* D = (const float*)Db.buf;
  int64_t* as = (int64_t*)Ab.buf;
  mi = PyMem_Malloc(k * sizeof *mi);
  cnt = PyMem_Calloc(k + 1, sizeof *cnt);
  start = PyMem_Malloc((k + 1) * sizeof *start);
  mem = PyMem_Malloc(N * sizeof *mem);
  vals = PyMem_Malloc(k * sizeof *vals);
  intra = PyMem_Malloc(N * sizeof *intra);
  if (!mi || !cnt || !start || !mem || !vals || !intra) {
    PyErr_NoMemory();
    goto done;
  }
  for (Py_ssize_t j = 0; j < k; j++) {
    mi[j] = PyLong_AsSsize_t(PyList_GET_ITEM(med, j));
    if (mi[j] == -1 && PyErr_Occurred()) goto done;
    if (mi[j] < 0) mi[j] += N;  /* (numpy's negative index) */
    if (mi[j] < 0 || mi[j] >= N) {
      PyErr_SetString(PyExc_IndexError, "rmsdkey.kmed_step: medoid index out of range");
      goto done;
    }
  }
  for (Py_ssize_t i = 0; i < N; i++) {
    const float* row = D + i * N;
    for (Py_ssize_t j = 0; j < k; j++) vals[j] = row[mi[j]];
    as[i] = (int64_t)argmin_f32(vals, k);
    cnt[as[i] + 1]++;
  }
  start[0] = 0;
  for (Py_ssize_t j = 0; j < k; j++) start[j + 1] = start[j] + cnt[j + 1];
  for (Py_ssize_t j = 0; j <= k; j++) cnt[j] = start[j];
  for (Py_ssize_t i = 0; i < N; i++) mem[cnt[as[i]]++] = i;  /* (np.where order: ascending) */
  out = PyList_New(k);
  for (Py_ssize_t j = 0; out && j < k; j++) {
    const Py_ssize_t n = start[j + 1] - start[j];
    Py_ssize_t pick = -1;
    if (n) {
      const Py_ssize_t* ix = mem + start[j];
      for (Py_ssize_t a = 0; a < n; a++) intra[a] = pw_sum(D + ix[a] * N, ix, n);
      pick = ix[argmin_f32(intra, n)];
    }
    PyObject* v = PyLong_FromSsize_t(pick);
    if (!v) {
      Py_CLEAR(out);
      break;
    }
    PyList_SET_ITEM(out, j, v);
  }
done:
  PyMem_Free(mi);
  PyMem_Free(cnt);
  PyMem_Free(start);
  PyMem_Free(mem);
  PyMem_Free(vals);
  PyMem_Free(intra);
  PyBuffer_Release(&Db);
  PyBuffer_Release(&Ab);
  return out;
}


static PyMethodDef METHODS[] = {
                                {"key", key, METH_VARARGS, "the pair key string of a span (RmsdBPE._pair_key)"},
                                {"pack", pack, METH_VARARGS, "whole-residue span geometry, geobpe_nerf layout"},
                                {"reprs", reprs, METH_VARARGS, "repr(float) of each value (test)"},
                                {"setgeo", setgeo, METH_VARARGS, "set_token_geo into the chain's column lists"},
                                {"merge", merge, METH_VARARGS, "the occurrence loop of a merge (RmsdBPE._merge)"},
                                {"memo_new", memo_new, METH_NOARGS, "a new pair-key memo (merge's 7th state item)"},
                                {"memo_len", memo_len, METH_O, "keys in a pair-key memo"},
                                {"memo_check", memo_check, METH_VARARGS,
                                 "memo_check(on) -> memo hits compared since the last call (test)"},
                                {"prio", prio, METH_VARARGS, "the priority updates of a merge (RmsdBPE._merge)"},
                                {"rekey", rekey, METH_VARARGS, "the re-keying after a glue re-optimisation (RmsdBPE._merge)"},
                                {"packc", packc, METH_VARARGS, "pack() with spans as (chain, q, r)"},
                                {"kmed_step", kmed_step, METH_VARARGS, "one k-medoids iteration (algo.py:191-213)"},
                                {"packa", packa, METH_VARARGS, "pack() with spans as an int64 (n, 3) buffer"},
                                {"spans_occ", spans_occ, METH_VARARGS, "the spans of a key's occurrences"},
                                {NULL, NULL, 0, NULL}};
static struct PyModuleDef MOD = {PyModuleDef_HEAD_INIT, "_rmsdkey", NULL, -1, METHODS, NULL, NULL, NULL, NULL};
PyMODINIT_FUNC PyInit__rmsdkey(void) {
  for (int i = 0; i < A_COUNT; i++)
    if (!ATTR[i] && !(ATTR[i] = PyUnicode_InternFromString(ATTR_NAMES[i]))) return NULL;
  for (int i = 0; i < 9; i++)
    if (!PACK_KEYS[i] && !(PACK_KEYS[i] = PyUnicode_InternFromString(PACK_NAMES[i]))) return NULL;
  for (int i = 0; i < 9; i++)
    if (!NAME_KEYS[i] && !(NAME_KEYS[i] = PyUnicode_InternFromString(NAMES[i]))) return NULL;
  return PyModule_Create(&MOD);
}
