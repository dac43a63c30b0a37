/* dadmm_ingest.c — native graph ingestion (CPython extension module dadmm_hip._ingest).
 *
 * Replaces the host side of compute_sum_neighbors (unfolded_DLASSO.py:111-118) and the graph walk
 * of compute_delta (:127-140) for a batch of networkx graphs: one C pass over every graph's
 * adjacency dict (graph._adj, whose iteration order is graph.neighbors(p)) builds, per sample s
 * and agent p,
 *   nbr[s][p]   uint64 neighbour mask (bit q <=> q in graph.neighbors(p)),
 *   deg[s][p]   float len(neighbors(p)),
 *   order[s][p] the adjacency order packed 4 bits per neighbour (first 8 neighbours),
 *   the visit list of agent p: the ids q whose term (y_p - y_q) compute_delta adds to delta[p],
 *     in its order — q < p with p in neighbors(q) (ascending), then neighbors(p) in adjacency
 *     order (a self-loop twice), then q > p with p in neighbors(q) (ascending),
 * exactly as dadmm_hip.graph._visit_lists does in Python. The Python per-graph loops were the
 * dominant host cost of a forward over thousands of distinct graphs (missing #4).
 *
 * batch(graph_list, P) -> (nbr, deg, order, vptr, vq as bytearrays, ascending, symmetric)
 * Raises ValueError for a neighbour id outside 0..P-1 (the reference would index past the
 * state), TypeError for a graph without a dict adjacency (the caller then takes the Python path).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAXP 64

/* Node ids are small ints, which CPython keeps as singletons in one contiguous array: an id key
 * is recognised by its address (checked against the singletons of 0..P-1), anything else goes
 * through PyLong_AsLong. */
static long key_id(PyObject* k, PyObject* const* small, int P) {
    const char* a = (const char*)k;
    const char* b = (const char*)small[0];
    const ptrdiff_t st = (const char*)small[1] - b;
    if (st > 0 && a >= b) {
        const ptrdiff_t d = a - b;
        if (d % st == 0 && d / st < P && (PyObject*)k == small[d / st]) return (long)(d / st);
    }
    return PyLong_AsLong(k);
}

static PyObject* batch(PyObject* self, PyObject* args) {
    (void)self;
    PyObject* glist;
    int P;
    if (!PyArg_ParseTuple(args, "Oi", &glist, &P)) return NULL;
    if (P < 1 || P > MAXP) {
        PyErr_Format(PyExc_ValueError, "P=%d: 1 <= P <= %d", P, MAXP);
        return NULL;
    }
    PyObject* seq = PySequence_Fast(glist, "graph_list must be a sequence");
    if (!seq) return NULL;
    const Py_ssize_t B = PySequence_Fast_GET_SIZE(seq);
    PyObject** items = PySequence_Fast_ITEMS(seq);
    const size_t BP = (size_t)B * P;

    uint64_t* nbr = (uint64_t*)calloc(BP ? BP : 1, sizeof(uint64_t));
    float* deg = (float*)calloc(BP ? BP : 1, sizeof(float));
    uint32_t* order = (uint32_t*)calloc(BP ? BP : 1, sizeof(uint32_t));
    int32_t* vptr = (int32_t*)calloc(BP + 1, sizeof(int32_t));
    /* own adjacency lists in order, for the second pass: at most P entries each (distinct keys) */
    uint8_t* own = (uint8_t*)malloc(BP ? BP * P : 1);
    uint8_t* ownlen = (uint8_t*)calloc(BP ? BP : 1, 1);
    uint8_t* vq = NULL;
    PyObject* adj_name = PyUnicode_InternFromString("_adj");
    PyObject* out = NULL;
    int ascending = 1, symmetric = 1;
    PyObject* small[MAXP + 1];
    for (int q = 0; q <= MAXP; ++q) small[q] = PyLong_FromLong(q);   /* singletons: borrowed back */
    for (int q = 0; q <= MAXP; ++q) Py_DECREF(small[q]);
    if (!nbr || !deg || !order || !vptr || !own || !ownlen || !adj_name) {
        PyErr_NoMemory();
        goto done;
    }

    for (Py_ssize_t s = 0; s < B; ++s) {
        PyObject* adj = PyObject_GetAttr(items[s], adj_name);   /* new reference */
        if (!adj || !PyDict_Check(adj)) {
            Py_XDECREF(adj);
            PyErr_Clear();
            PyErr_SetString(PyExc_TypeError, "graph without a dict adjacency (_adj)");
            goto done;
        }
        for (int p = 0; p < P; ++p) {
            PyObject* nb = PyDict_GetItemWithError(adj, small[p]);   /* borrowed */
            if (!nb) {
                if (!PyErr_Occurred())
                    PyErr_Format(PyExc_KeyError, "graph %zd has no node %d", s, p);
                Py_DECREF(adj);
                goto done;
            }
            if (!PyDict_Check(nb)) {
                PyErr_SetString(PyExc_TypeError, "adjacency rows must be dicts");
                Py_DECREF(adj);
                goto done;
            }
            const size_t sp = (size_t)s * P + p;
            Py_ssize_t pos = 0;
            PyObject *qk, *qv;
            int t = 0, prev = -1;
            uint64_t m = 0;
            uint32_t ord = 0;
            while (PyDict_Next(nb, &pos, &qk, &qv)) {
                const long q = key_id(qk, small, P);
                if (q == -1 && PyErr_Occurred()) {
                    Py_DECREF(adj);
                    goto done;
                }
                if (q < 0 || q >= P) {
                    PyErr_Format(PyExc_ValueError, "neighbour id %ld of agent %d: must be an agent 0..%d",
                                 q, p, P - 1);
                    Py_DECREF(adj);
                    goto done;
                }
                if (t >= P) {   /* distinct keys in 0..P-1: cannot happen */
                    PyErr_SetString(PyExc_ValueError, "adjacency row longer than P");
                    Py_DECREF(adj);
                    goto done;
                }
                m |= (uint64_t)1 << q;
                if (t < 8) ord |= (uint32_t)(q & 15) << (4 * t);
                if (q <= prev) ascending = 0;
                prev = (int)q;
                own[sp * P + t] = (uint8_t)q;
                ++t;
            }
            nbr[sp] = m;
            deg[sp] = (float)t;
            order[sp] = ord;
            ownlen[sp] = (uint8_t)t;
        }
        Py_DECREF(adj);
    }

    /* visit lists: into[p] = {p' : p in N(p')} from the masks (general: also directed graphs) */
    {
        size_t total = 0;
        uint64_t* intos = (uint64_t*)calloc(BP ? BP : 1, sizeof(uint64_t));
        if (!intos) {
            PyErr_NoMemory();
            goto done;
        }
        for (Py_ssize_t s = 0; s < B; ++s) {   /* transpose each sample's bit matrix, O(edges) */
            const uint64_t* ms = nbr + (size_t)s * P;
            uint64_t* in = intos + (size_t)s * P;
            for (int pp = 0; pp < P; ++pp)
                for (uint64_t m = ms[pp] & ~((uint64_t)1 << pp); m; m &= m - 1)
                    in[__builtin_ctzll(m)] |= (uint64_t)1 << pp;
        }
        for (Py_ssize_t s = 0; s < B; ++s) {
            const uint64_t* ms = nbr + (size_t)s * P;
            for (int p = 0; p < P; ++p) {
                const uint64_t into = intos[(size_t)s * P + p];
                if (into != (ms[p] & ~((uint64_t)1 << p))) symmetric = 0;
                const int loop = (int)((ms[p] >> p) & 1u);
                const size_t c = (size_t)__builtin_popcountll(into) + ownlen[(size_t)s * P + p] + loop;
                total += c;
                vptr[(size_t)s * P + p + 1] = (int32_t)total;
                if (total >= ((size_t)1 << 31)) {
                    free(intos);
                    PyErr_SetString(PyExc_ValueError, "visit lists past 2^31 entries (split the batch)");
                    goto done;
                }
            }
        }
        vq = (uint8_t*)malloc(total ? total : 1);
        if (!vq) {
            free(intos);
            PyErr_NoMemory();
            goto done;
        }
        for (size_t sp = 0; sp < BP; ++sp) {
            const int p = (int)(sp % (size_t)P);
            uint8_t* o = vq + vptr[sp];
            const uint64_t into = intos[sp];
            const uint64_t below = p ? into & (~(uint64_t)0 >> (64 - p)) : 0;
            for (uint64_t m = below; m; m &= m - 1) *o++ = (uint8_t)__builtin_ctzll(m);
            const uint8_t* ol = own + sp * P;
            for (int t = 0; t < ownlen[sp]; ++t) {
                *o++ = ol[t];
                if (ol[t] == p) *o++ = ol[t];   /* a self-loop's += and -= */
            }
            for (uint64_t m = into & ~below & ~((uint64_t)1 << p); m; m &= m - 1)
                *o++ = (uint8_t)__builtin_ctzll(m);
        }
        free(intos);
        /* bytearrays: numpy views of them are writable (torch.from_numpy warns on read-only ones) */
        out = Py_BuildValue("(NNNNNNN)", PyByteArray_FromStringAndSize((const char*)nbr, (Py_ssize_t)(BP * 8)),
                            PyByteArray_FromStringAndSize((const char*)deg, (Py_ssize_t)(BP * 4)),
                            PyByteArray_FromStringAndSize((const char*)order, (Py_ssize_t)(BP * 4)),
                            PyByteArray_FromStringAndSize((const char*)vptr, (Py_ssize_t)((BP + 1) * 4)),
                            PyByteArray_FromStringAndSize((const char*)vq, (Py_ssize_t)total),
                            PyBool_FromLong(ascending), PyBool_FromLong(symmetric));
    }

done:
    Py_XDECREF(adj_name);
    free(nbr);
    free(deg);
    free(order);
    free(vptr);
    free(own);
    free(ownlen);
    free(vq);
    Py_DECREF(seq);
    return out;
}

static PyMethodDef methods[] = {
    {"batch", batch, METH_VARARGS,
     "batch(graph_list, P) -> (nbr, deg, order, vptr, vq, ascending, symmetric) as bytearrays / bools"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_ingest",
                                    "native graph ingestion (dadmm_hip.graph)", -1, methods};

PyMODINIT_FUNC PyInit__ingest(void) { return PyModule_Create(&module); }
