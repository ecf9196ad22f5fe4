/*
 * rt_host.c — C host library around the render call (include/rt/host.h):
 * camera set-up, OBJ/MTL/PPM loading and PPM output with the reference's
 * data model (triangle / material / texel-table layout).
 *
 * Loader semantics follow mesh.h:96-234 / texture.h:175-354 / rtutility.h:
 * 233-290 where those are well defined, and fix what crashes there
 * (SURVEY.md §7 "Loader gaps"): `f v//vn` and `f v` faces, n-gons (first
 * three vertices as the reference's sscanf keeps them, or a fan), CRLF
 * files, MTL materials with Kd but no map_Kd, and missing files (errors
 * instead of NULL dereferences).
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt/host.h"
#include "rt/rt.h"

/* ---- camera.h:21-40 ------------------------------------------------------ */
static rt_vec3 v3(double a, double b, double c) { rt_vec3 r = {{a, b, c}}; return r; }
static rt_vec3 vsub(rt_vec3 a, rt_vec3 b) { return v3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
static rt_vec3 vadd(rt_vec3 a, rt_vec3 b) { return v3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
static rt_vec3 vmul(rt_vec3 a, double t) { return v3(a.e[0] * t, a.e[1] * t, a.e[2] * t); }
static rt_vec3 vdiv(rt_vec3 a, double t) { return v3(a.e[0] / t, a.e[1] / t, a.e[2] / t); }
static rt_vec3 vcross(rt_vec3 u, rt_vec3 v)
{
    return v3(u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2],
              u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
static rt_vec3 vnorm(rt_vec3 a)
{
    return vdiv(a, sqrt(a.e[0] * a.e[0] + a.e[1] * a.e[1] + a.e[2] * a.e[2]));
}

rt_camera rt_host_init_camera(rt_point3 origin, rt_point3 target, rt_vec3 up, double vfov, double ratio)
{
    rt_camera cam;
    double theta = vfov * 3.1415926535897932385 / 180.0;   /* degrees_to_radians, camera.h:17-19 */
    double h = tan(theta / 2);
    double hauteur_viewport = 2.0 * h;
    double largeur_viewport = ratio * hauteur_viewport;
    rt_vec3 w = vnorm(vsub(origin, target));
    rt_vec3 u = vnorm(vcross(up, w));
    rt_vec3 v = vcross(w, u);
    cam.origin = origin;
    cam.horizontal = vmul(u, largeur_viewport);
    cam.vertical = vmul(v, hauteur_viewport);
    cam.coin_bas_gauche = vsub(cam.origin, vadd(vdiv(cam.horizontal, 2), vadd(vdiv(cam.vertical, 2), w)));
    return cam;
}

void rt_host_move_mesh(double x, double y, double z, rt_triangle* t, int n)
{
    for (int i = 0; i < n; i++) {           /* mesh.h:220-234 */
        t[i].A.e[0] += x; t[i].B.e[0] += x; t[i].C.e[0] += x;
        t[i].A.e[1] += y; t[i].B.e[1] += y; t[i].C.e[1] += y;
        t[i].A.e[2] += z; t[i].B.e[2] += z; t[i].C.e[2] += z;
    }
}

void rt_host_free(void* p) { free(p); }

void rt_host_cuda_materials(rt_mesh* m)
{
    if (!m || !m->triangles || !m->quelMatPourTri) return;
    for (int i = 0; i < m->nbTriangles; i++) {
        const int k = m->quelMatPourTri[i];
        rt_material* mt = &m->triangles[i].mat;
        memset(mt, 0, sizeof *mt);
        if (k < 0 || k >= m->nbMaterials) continue;
        for (int a = 0; a < 3; a++) mt->diffuseColor.e[a] = (double)(float)(m->kd ? m->kd[k].e[a] : 0.0);
        const float shininess = (float)(m->ns ? m->ns[k] : 0.0);
        mt->reflectionStrength = (double)(shininess / 100);     /* triangle.hu:104 */
        mt->alpha = 1.0;
    }
}

/* ---- growable arrays ----------------------------------------------------- */
typedef struct { void* p; size_t n, cap, sz; } vec_t;
static int vpush(vec_t* v, const void* x)
{
    if (v->n == v->cap) {
        size_t c = v->cap ? v->cap * 2 : 64;
        void* q = realloc(v->p, c * v->sz);
        if (!q) return RT_ENOMEM;
        v->p = q;
        v->cap = c;
    }
    memcpy((char*)v->p + v->n * v->sz, x, v->sz);
    v->n++;
    return RT_OK;
}

static void rstrip(char* s)
{
    size_t n = strlen(s);
    while (n && (s[n - 1] == '\n' || s[n - 1] == '\r' || s[n - 1] == ' ' || s[n - 1] == '\t')) s[--n] = 0;
}
static char* lskip(char* s)
{
    while (*s == ' ' || *s == '\t') s++;
    return s;
}

/* ---- MTL ----------------------------------------------------------------- */
typedef struct { char* name; char* map_kd; rt_vec3 kd; double ns; } mtl_rec;

static int parse_mtl(const char* path, mtl_rec** out, int* n_out)
{
    *out = NULL;
    *n_out = 0;
    FILE* f = fopen(path, "r");
    if (!f) return RT_EINVAL;
    vec_t v = {NULL, 0, 0, sizeof(mtl_rec)};
    char line[4096];
    mtl_rec* cur = NULL;
    char* dir = strdup(path);
    char* slash = strrchr(dir, '/');
    if (slash) slash[1] = 0; else dir[0] = 0;
    while (fgets(line, sizeof line, f)) {
        rstrip(line);
        char* s = lskip(line);
        if (!strncmp(s, "newmtl", 6) && isspace((unsigned char)s[6])) {
            mtl_rec r;
            memset(&r, 0, sizeof r);
            r.name = strdup(lskip(s + 6));
            if (vpush(&v, &r)) break;
            cur = (mtl_rec*)v.p + (v.n - 1);
        } else if (cur && !strncmp(s, "map_Kd", 6) && isspace((unsigned char)s[6])) {
            char* p = lskip(s + 6);
            if (!strncmp(p, "./", 2)) p += 2;      /* rtutility.h:266-268 */
            free(cur->map_kd);
            cur->map_kd = (char*)malloc(strlen(dir) + strlen(p) + 1);
            strcpy(cur->map_kd, dir);
            strcat(cur->map_kd, p);
        } else if (cur && s[0] == 'K' && s[1] == 'd' && isspace((unsigned char)s[2])) {
            sscanf(s + 2, "%lf %lf %lf", &cur->kd.e[0], &cur->kd.e[1], &cur->kd.e[2]);
        } else if (cur && s[0] == 'N' && s[1] == 's' && isspace((unsigned char)s[2])) {
            sscanf(s + 2, "%lf", &cur->ns);
        }
    }
    free(dir);
    fclose(f);
    *out = (mtl_rec*)v.p;
    *n_out = (int)v.n;
    return RT_OK;
}

static void free_mtl(mtl_rec* r, int n)
{
    for (int i = 0; i < n; i++) {
        free(r[i].name);
        free(r[i].map_kd);
    }
    free(r);
}

/* ---- OBJ ----------------------------------------------------------------- */
/* parse one face vertex "v", "v/vt", "v/vt/vn" or "v//vn" */
static int parse_fv(const char* tok, int* vi, int* ti)
{
    char* end;
    long a = strtol(tok, &end, 10);
    if (end == tok) return 0;
    *vi = (int)a;
    *ti = 0;
    if (*end == '/') {
        const char* q = end + 1;
        if (*q != '/') {
            long b = strtol(q, &end, 10);
            if (end != q) *ti = (int)b;
        }
    }
    return 1;
}

static int fix_index(int idx, size_t n)
{
    if (idx < 0) return (int)n + idx;   /* relative index */
    return idx - 1;
}

int rt_host_load_obj(const char* obj_path, const char* mtl_path, int ngon_mode, rt_mesh* out)
{
    if (!obj_path || !out) return RT_EINVAL;
    memset(out, 0, sizeof *out);
    FILE* f = fopen(obj_path, "r");
    if (!f) return RT_EINVAL;
    mtl_rec* mtl = NULL;
    int nmtl = 0;
    if (mtl_path) parse_mtl(mtl_path, &mtl, &nmtl);   /* missing MTL: materials without maps */

    vec_t V = {NULL, 0, 0, sizeof(rt_vec3)}, T = {NULL, 0, 0, sizeof(rt_uv)};
    vec_t tris = {NULL, 0, 0, sizeof(rt_triangle)}, qm = {NULL, 0, 0, sizeof(int)};
    vec_t names = {NULL, 0, 0, sizeof(char*)};
    int rc = RT_OK, cur_mat = -1;
    char line[8192];
    while (rc == RT_OK && fgets(line, sizeof line, f)) {
        rstrip(line);
        char* s = line;
        if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
            rt_vec3 p = v3(0, 0, 0);
            sscanf(s + 2, "%lf %lf %lf", &p.e[0], &p.e[1], &p.e[2]);
            rc = vpush(&V, &p);
        } else if (s[0] == 'v' && s[1] == 't' && (s[2] == ' ' || s[2] == '\t')) {
            rt_uv t = {0, 0};
            sscanf(s + 3, "%lf %lf", &t.u, &t.v);
            rc = vpush(&T, &t);
        } else if (!strncmp(s, "usemtl", 6)) {    /* mesh.h:176-182: one material per usemtl line */
            char* nm = strdup(lskip(s + 6));
            rc = vpush(&names, &nm);
            cur_mat++;
        } else if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
            int vi[64], ti[64], nv = 0;
            char* save = NULL;
            for (char* tok = strtok_r(s + 2, " \t", &save); tok && nv < 64; tok = strtok_r(NULL, " \t", &save))
                if (parse_fv(tok, &vi[nv], &ti[nv])) nv++;
            if (nv < 3) continue;
            if (cur_mat < 0) { rc = RT_EINVAL; break; }   /* face before any usemtl: reference index -1 */
            int ntri = (ngon_mode == RT_OBJ_FAN_QUADS) ? nv - 2 : 1;
            for (int k = 0; k < ntri; k++) {
                int c[3] = {0, k + 1, k + 2};
                rt_triangle tr;
                memset(&tr, 0, sizeof tr);
                rt_vec3* P[3] = {&tr.A, &tr.B, &tr.C};
                rt_uv* U[3] = {&tr.uvA, &tr.uvB, &tr.uvC};
                for (int q = 0; q < 3; q++) {
                    int a = fix_index(vi[c[q]], V.n);
                    if (a < 0 || (size_t)a >= V.n) { rc = RT_EINVAL; break; }
                    *P[q] = ((rt_vec3*)V.p)[a];
                    if (ti[c[q]]) {
                        int b = fix_index(ti[c[q]], T.n);
                        if (b < 0 || (size_t)b >= T.n) { rc = RT_EINVAL; break; }
                        *U[q] = ((rt_uv*)T.p)[b];
                    }
                }
                if (rc) break;
                /* mesh.h:206: (material){SKY, BLACK, 0.0, 0.0} */
                tr.mat.diffuseColor = v3(0.784, 0.965, 1);
                if ((rc = vpush(&tris, &tr)) || (rc = vpush(&qm, &cur_mat))) break;
            }
        }
    }
    fclose(f);
    free(V.p);
    free(T.p);
    if (rc == RT_OK) {
        out->triangles = (rt_triangle*)tris.p;
        out->nbTriangles = (int)tris.n;
        out->quelMatPourTri = (int*)qm.p;
        out->nbMaterials = (int)names.n;
        out->material_names = (char**)names.p;
        out->texture_paths = (char**)calloc(names.n ? names.n : 1, sizeof(char*));
        out->kd = (rt_vec3*)calloc(names.n ? names.n : 1, sizeof(rt_vec3));
        out->ns = (double*)calloc(names.n ? names.n : 1, sizeof(double));
        for (size_t k = 0; k < names.n; k++) {
            const char* nm = out->material_names[k];
            for (int j = 0; j < nmtl; j++) {
                if (!strcmp(mtl[j].name, nm)) {
                    if (mtl[j].map_kd) out->texture_paths[k] = strdup(mtl[j].map_kd);
                    out->kd[k] = mtl[j].kd;
                    out->ns[k] = mtl[j].ns;
                    break;
                }
            }
        }
    } else {
        free(tris.p);
        free(qm.p);
        for (size_t k = 0; k < names.n; k++) free(((char**)names.p)[k]);
        free(names.p);
    }
    free_mtl(mtl, nmtl);
    return rc;
}

void rt_host_free_mesh(rt_mesh* m)
{
    if (!m) return;
    for (int k = 0; k < m->nbMaterials; k++) {
        if (m->material_names) free(m->material_names[k]);
        if (m->texture_paths) free(m->texture_paths[k]);
    }
    free(m->material_names);
    free(m->texture_paths);
    free(m->kd);
    free(m->ns);
    free(m->triangles);
    free(m->quelMatPourTri);
    memset(m, 0, sizeof *m);
}

/* ---- PPM ----------------------------------------------------------------- */
static int next_token(FILE* f, char* buf, size_t n)
{
    int c;
    for (;;) {
        c = fgetc(f);
        if (c == EOF) return 0;
        if (c == '#') {
            while (c != '\n' && c != EOF) c = fgetc(f);
            continue;
        }
        if (!isspace(c)) break;
    }
    size_t k = 0;
    while (c != EOF && !isspace(c) && k + 1 < n) {
        buf[k++] = (char)c;
        c = fgetc(f);
    }
    buf[k] = 0;
    return 1;
}

int rt_host_read_ppm(const char* path, int* w, int* h, int* maxval, int** values)
{
    if (!path || !w || !h || !maxval || !values) return RT_EINVAL;
    *values = NULL;
    FILE* f = fopen(path, "r");
    if (!f) return RT_EINVAL;
    char tok[64];
    int rc = RT_EINVAL;
    if (next_token(f, tok, sizeof tok) && !strcmp(tok, "P3") && next_token(f, tok, sizeof tok) &&
        (*w = atoi(tok)) > 0 && next_token(f, tok, sizeof tok) && (*h = atoi(tok)) > 0 &&
        next_token(f, tok, sizeof tok) && (*maxval = atoi(tok)) > 0) {
        size_t n = (size_t)*w * (size_t)*h * 3;
        int* v = (int*)malloc(n * sizeof(int));
        if (!v) {
            fclose(f);
            return RT_ENOMEM;
        }
        size_t k = 0;
        while (k < n && next_token(f, tok, sizeof tok)) v[k++] = atoi(tok);
        if (k == n) {
            *values = v;
            rc = RT_OK;
        } else {
            free(v);
        }
    }
    fclose(f);
    return rc;
}

int rt_host_write_ppm(const char* path, const rt_color* canva, int W, int H)
{
    if (!path || !canva || W < 1 || H < 1) return RT_EINVAL;
    FILE* f = fopen(path, "w");
    if (!f) return RT_EINVAL;
    fprintf(f, "P3\n%d %d\n255\n", W, H);
    for (int j = H - 1; j >= 0; j--)
        for (int i = 0; i < W; i++) {
            const rt_color* c = &canva[(size_t)j * W + i];
            fprintf(f, "%d %d %d\n", (int)(c->e[0]), (int)(c->e[1]), (int)(c->e[2]));
        }
    return fclose(f) == 0 ? RT_OK : RT_EINVAL;
}

/* ---- texel table, texture.h:175-354 --------------------------------------- */
static char* with_suffix(const char* tex_png, const char* suffix)
{
    const char* pos = strstr(tex_png, ".png");
    size_t len = pos ? (size_t)(pos - tex_png) : strlen(tex_png);
    char* s = (char*)malloc(len + strlen(suffix) + 1);
    memcpy(s, tex_png, len);
    strcpy(s + len, suffix);
    return s;
}

int rt_host_load_textures(const rt_mesh* mesh, int kd_fallback, rt_material** mat_list, int* tw, int* th)
{
    if (!mesh || !mat_list || !tw || !th) return RT_EINVAL;
    *mat_list = NULL;
    int n = mesh->nbMaterials;
    if (n < 1) return RT_EINVAL;
    int W = 0, H = 0;
    int** rgb = (int**)calloc((size_t)n, sizeof(int*));
    int** alp = (int**)calloc((size_t)n, sizeof(int*));
    int* mv = (int*)calloc((size_t)n, sizeof(int));
    int* ma = (int*)calloc((size_t)n, sizeof(int));
    int rc = RT_OK;
    for (int k = 0; k < n && rc == RT_OK; k++) {
        const char* p = mesh->texture_paths ? mesh->texture_paths[k] : NULL;
        if (!p) {
            if (!kd_fallback) rc = RT_EINVAL;
            continue;
        }
        char* tp = with_suffix(p, ".ppm");
        char* ap = with_suffix(p, "_alpha.ppm");
        int w1, h1, w2, h2;
        rc = rt_host_read_ppm(tp, &w1, &h1, &mv[k], &rgb[k]);
        if (rc == RT_OK) rc = rt_host_read_ppm(ap, &w2, &h2, &ma[k], &alp[k]);
        if (rc == RT_OK && (w1 != w2 || h1 != h2)) rc = RT_EINVAL;
        if (rc == RT_OK && W && (w1 != W || h1 != H)) rc = RT_EINVAL;   /* one size for all (texture.h:305) */
        W = w1;
        H = h1;
        free(tp);
        free(ap);
    }
    if (rc == RT_OK) {
        if (!W) W = H = 1;
        size_t plane = (size_t)W * H;
        rt_material* m = (rt_material*)calloc(plane * (size_t)n, sizeof(rt_material));
        if (!m) rc = RT_ENOMEM;
        for (int k = 0; rc == RT_OK && k < n; k++) {
            rt_material* base = m + plane * (size_t)k;
            if (!rgb[k]) {        /* Kd-flat material (triangle.hu:104-105 semantics) */
                float shin = (float)mesh->ns[k];
                for (size_t q = 0; q < plane; q++) {
                    base[q].diffuseColor = mesh->kd[k];
                    base[q].alpha = 1.0;
                    base[q].reflectionStrength = (double)(shin / 100);
                }
                continue;
            }
            /* rows bottom-up: file row r (top first) -> table row H-1-r */
            for (int i = H - 1, r = 0; i >= 0; i--, r++)
                for (int j = 0; j < W; j++) {
                    size_t idx = (size_t)i * W + j;
                    const int* px = rgb[k] + ((size_t)r * W + j) * 3;
                    const int* pa = alp[k] + ((size_t)r * W + j) * 3;
                    base[idx].diffuseColor = v3((double)px[0] / mv[k], (double)px[1] / mv[k], (double)px[2] / mv[k]);
                    base[idx].alpha = (double)pa[0] / ma[k];
                    base[idx].emissionStrength = 0.0;
                }
        }
        if (rc == RT_OK) {
            *mat_list = m;
            *tw = W;
            *th = H;
        } else {
            free(m);
        }
    }
    for (int k = 0; k < n; k++) {
        free(rgb[k]);
        free(alp[k]);
    }
    free(rgb);
    free(alp);
    free(mv);
    free(ma);
    return rc;
}
