/*
 * xf_analysis.c — offline study of transform drift in mixed worlds (final_scene), CPU only.
 *
 * Built as a unity build over the oracle (tools only, never shipped):
 *   gcc -O2 -fopenmp -ffp-contract=off -Iinclude -shared -fPIC tools/xf_analysis.c -o /tmp/libxf.so -lm
 * For every ray the reference's hit() receives on a sample of pixels, it reports:
 *   - the reference walk's visits, split into the "top" part (nodes whose subtree holds a transform)
 *     and the transform-free subtrees (TF) entered from it (macro leaves),
 *   - how many transform chains the walk entered (K, the number of in-place drifts),
 *   - whether the ray's line (tmax = inf) meets any box of a BVH node with a transform child.
 */
#include "../oracle/oracle_rt.c"

#include <stdio.h>

static uint8_t *g_tf;       /* per record: 1 = subtree holds no translate / rotate */
static uint8_t *g_xfpar;
static int g_dedup = 0;
static rtr_aabb *g_xfbox;   /* per record: union of the boxes of the BVH leaves with a transform child below it */
static uint8_t *g_hasxf;    /* per record: g_xfbox valid (a transform chain below) */
static uint32_t *g_nprims;
static uint32_t g_dyn_min = 0;   /* dynamic collapse only for top nodes with at least this many TF prims */  /* per record: transform-free prims below (chains excluded) */    /* per record: 1 = BVH node with a transform child */

static int tf_of(const rt_scene *sc, uint16_t r) {
  if (g_tf[r] != 2) return g_tf[r];
  const rtr_hittable *h = &sc->hittables[r];
  int v = 1;
  switch (h->kind) {
    case RTR_OBJ_BVH: {
      uint16_t l = sc->refs[h->u.bvh.left], rr = sc->refs[h->u.bvh.right];
      int a = tf_of(sc, l), b = tf_of(sc, rr);
      v = a && b;
      int kl = sc->hittables[l].kind, kr = sc->hittables[rr].kind;
      g_xfpar[r] = (kl == RTR_OBJ_TRANSLATE || kl == RTR_OBJ_YROTATE || kr == RTR_OBJ_TRANSLATE || kr == RTR_OBJ_YROTATE);
    } break;
    case RTR_OBJ_GROUP:
      for (uint16_t i = 0; i < h->u.group.count; ++i) v &= tf_of(sc, (uint16_t)(h->u.group.first + i));
      break;
    case RTR_OBJ_TRANSLATE: case RTR_OBJ_YROTATE: v = 0; break;
    default: v = 1;
  }
  g_tf[r] = (uint8_t)v;
  return v;
}

static void xfbox_of(const rt_scene *sc, uint16_t r) {
  const rtr_hittable *h = &sc->hittables[r];
  if (g_hasxf[r] != 2) return;
  g_hasxf[r] = 0; g_nprims[r] = 0;
  rtr_aabb b = {INFINITY, -INFINITY, INFINITY, -INFINITY, INFINITY, -INFINITY};
  int has = 0;
  uint32_t np = 0;
  if (h->kind == RTR_OBJ_BVH) {
    if (g_xfpar[r]) { b = h->u.bvh.box; has = 1; }
    uint16_t ch[2] = {sc->refs[h->u.bvh.left], sc->refs[h->u.bvh.right]};
    for (int k = 0; k < (ch[0] == ch[1] ? 1 : 2); ++k) {
      uint16_t c = ch[k];
      xfbox_of(sc, c);
      np += g_nprims[c];
      if (g_hasxf[c]) { rtr_aabb cb = g_xfbox[c]; has = 1;
        b.x0 = fminf(b.x0, cb.x0); b.x1 = fmaxf(b.x1, cb.x1); b.y0 = fminf(b.y0, cb.y0); b.y1 = fmaxf(b.y1, cb.y1);
        b.z0 = fminf(b.z0, cb.z0); b.z1 = fmaxf(b.z1, cb.z1); }
    }
  } else if (h->kind == RTR_OBJ_GROUP) {
    for (uint16_t i = 0; i < h->u.group.count; ++i) { uint16_t c = (uint16_t)(h->u.group.first + i); xfbox_of(sc, c); np += g_nprims[c];
      if (g_hasxf[c]) { rtr_aabb cb = g_xfbox[c]; has = 1;
        b.x0 = fminf(b.x0, cb.x0); b.x1 = fmaxf(b.x1, cb.x1); b.y0 = fminf(b.y0, cb.y0); b.y1 = fmaxf(b.y1, cb.y1);
        b.z0 = fminf(b.z0, cb.z0); b.z1 = fmaxf(b.z1, cb.z1); } }
  } else if (h->kind == RTR_OBJ_TRANSLATE || h->kind == RTR_OBJ_YROTATE) {
    np = 0;
  } else np = 1;
  g_hasxf[r] = (uint8_t)has; g_xfbox[r] = b; g_nprims[r] = np;
}

static void dyn_walk(const rt_scene *sc, const ray_t *ray0, double *st);
enum { S_RAYS, S_VIS_ALL, S_VIS_TOP, S_VIS_TF, S_MACRO, S_K, S_K0, S_LINE_XF, S_PRIM_TOP, S_MACRO_PRIMS,
       S_LINE_XF_K0, S_DEDUP, S_DTOP, S_DMACRO, S_DMPRIMS, S_DSAH, S_DBVH, S_DBVHPASS, S_DCHAIN, S_DPRIM, S_DGROUP, S_DTOP_K0, S_DRAYS_K0, S_NSTAT };

/* the reference walk, instrumented: a node popped in the top part counts as top, a TF subtree root
 * popped from the top part counts as one macro entry and all its nodes as TF visits */
static void walk(const rt_scene *sc, const ray_t *ray0, double *st) {
  href_stack *s = (href_stack *)malloc(sizeof(href_stack));
  s->count = 0; s->max_seen = 0; s->overflow = 0;
  ray_t ray = *ray0;
  float tmin = 0.001f, tmax = INFINITY;
  int tc = 0, yc = 0;
  /* per stack entry: 1 if it was pushed inside a TF subtree */
  static __thread uint8_t intf[STACK_CAP];
  uint16_t root = sc->refs[sc->root];
  s->data[s->count] = root; intf[s->count] = 0; s->count++;
  int K = 0;
  double dedup_saved = 0;
  double vis = 0, top = 0, tfv = 0, macro = 0, ptop = 0, mprims = 0;
  while (s->count > 0) {
    --s->count;
    uint16_t cur = s->data[s->count];
    int in_tf = intf[s->count];
    const rtr_hittable *h = &sc->hittables[cur];
    vis++;
    int child_tf = in_tf;
    if (!in_tf && g_tf[cur] && (h->kind == RTR_OBJ_BVH || h->kind == RTR_OBJ_GROUP)) { macro++; child_tf = 1; }
    if (in_tf || child_tf) { tfv++; if (h->kind != RTR_OBJ_BVH && h->kind != RTR_OBJ_GROUP) mprims++; }
    else { top++; if (h->kind == RTR_OBJ_SPHERE || h->kind == RTR_OBJ_QUAD || h->kind == RTR_OBJ_TRIANGLE) ptop++; }
#define PUSH(x) do { s->data[s->count] = (x); intf[s->count] = (uint8_t)child_tf; s->count++; } while (0)
    switch (h->kind) {
      case RTR_OBJ_SPHERE: {
        const rtr_sphere *sp = &h->u.sphere;
        vec3 center = line_at(sp->center, ray.time, sp->motion);
        vec3 oc = sub(center, ray.origin);
        float a = dot(ray.direction, ray.direction);
        float b = -2.0f * dot(ray.direction, oc);
        float c = dot(oc, oc) - sp->radius * sp->radius;
        float disc = b * b - 4 * a * c;
        if (disc >= 0) {
          float sq = sqrtf(disc);
          float rt = (-b - sq) / (2.0f * a);
          if (tmin >= rt || rt >= tmax) rt = (-b + sq) / (2.0f * a);
          if (tmin < rt && rt < tmax) tmax = rt;
        }
      } break;
      case RTR_OBJ_BVH: {
        const rtr_bvh *n = &h->u.bvh;
        if (aabb_hit(&n->box, &ray, tmin, tmax)) {
          uint16_t l = sc->refs[n->left], rr = sc->refs[n->right];
          if (l == rr && g_dedup && g_tf[l]) { dedup_saved += 1 + (sc->hittables[l].kind == RTR_OBJ_GROUP ? sc->hittables[l].u.group.count : 0); PUSH(l); }
          else { PUSH(rr); PUSH(l); }
        }
      } break;
      case RTR_OBJ_TRIANGLE: case RTR_OBJ_QUAD: {
        int tri = h->kind == RTR_OBJ_TRIANGLE;
        float al, be, t; vec3 p;
        plane_hit(&h->u.planar.geom, &ray, tmin, tmax, &al, &be, &t, &p);
        int inside = (0.0f <= al && al <= 1.0f) && (0.0f <= be && be <= 1.0f) && (!tri || al + be <= 1.0f);
        if (inside) tmax = t;
      } break;
      case RTR_OBJ_TRANSLATE: {
        const rtr_translate *tr = &h->u.translate;
        if (tc == 0) { ray.origin = sub(ray.origin, tr->offset); PUSH(cur); PUSH(tr->child); tc++; K++; }
        else { ray.origin = add(ray.origin, tr->offset); tc--; }
      } break;
      case RTR_OBJ_YROTATE: {
        const rtr_yrotate *y = &h->u.yrotate;
        float sn = y->sin_theta, cs = y->cos_theta;
        vec3 o = ray.origin, d = ray.direction;
        if (yc == 0) {
          ray.origin = v3((cs * o.x) - (sn * o.z), o.y, (sn * o.x) + (cs * o.z));
          ray.direction = v3((cs * d.x) - (sn * d.z), d.y, (sn * d.x) + (cs * d.z));
          PUSH(cur); PUSH(y->child); yc++;
        } else {
          ray.origin = v3((cs * o.x) + (sn * o.z), o.y, (-sn * o.x) + (cs * o.z));
          ray.direction = v3((cs * d.x) + (sn * d.z), d.y, (-sn * d.x) + (cs * d.z));
          yc--;
        }
      } break;
      case RTR_OBJ_GROUP:
        for (uint16_t i = 0; i < h->u.group.count; ++i) PUSH((uint16_t)(h->u.group.first + i));
        break;
    }
#undef PUSH
  }
  free(s);
  /* the line test: any transform-parent box met by the unmodified ray with tmax = inf */
  int line = 0;
  for (uint32_t r = 0; r < sc->hittable_count && !line; ++r)
    if (g_xfpar[r] && aabb_hit(&sc->hittables[r].u.bvh.box, ray0, tmin, INFINITY)) line = 1;
  st[S_RAYS] += 1; st[S_VIS_ALL] += vis; st[S_VIS_TOP] += top; st[S_VIS_TF] += tfv; st[S_MACRO] += macro;
  st[S_K] += K; st[S_K0] += (K == 0); st[S_LINE_XF] += line; st[S_PRIM_TOP] += ptop; st[S_MACRO_PRIMS] += mprims;
  st[S_LINE_XF_K0] += (line && K == 0);
  st[S_DEDUP] += dedup_saved;
  dyn_walk(sc, ray0, st);
}

/* counts only: the hybrid walk with dynamic collapse — a popped node whose subtree is transform-free, or
 * whose transform-leaf box union the ray misses (exact slab test, current tmax), is one macro (SAH walk
 * over its transform-free prims, cost estimated as 2 log2(n) + 4 steps); tmax updates come from the
 * reference walk of that subtree (same result) */
static void dyn_walk(const rt_scene *sc, const ray_t *ray0, double *st) {
  href_stack *s = (href_stack *)malloc(sizeof(href_stack));
  s->count = 0;
  ray_t ray = *ray0;
  float tmin = 0.001f, tmax = INFINITY;
  int tc = 0, yc = 0;
  static __thread uint8_t inm[STACK_CAP];
  s->data[s->count] = sc->refs[sc->root]; inm[s->count] = 0; s->count++;
  double top = 0, macro = 0, mprims = 0, sah = 0, nbvh = 0, nbvhpass = 0, nchain = 0, nprim = 0, ngroup = 0;
  int K = 0;
  while (s->count > 0) {
    --s->count;
    uint16_t cur = s->data[s->count];
    int in_m = inm[s->count];
    const rtr_hittable *h = &sc->hittables[cur];
    int child_m = in_m;
    if (!in_m) {
      top++;
      if (h->kind == RTR_OBJ_BVH) { nbvh++; if (aabb_hit(&h->u.bvh.box, &ray, tmin, tmax)) nbvhpass++; }
      else if (h->kind == RTR_OBJ_GROUP) ngroup++;
      else if (h->kind == RTR_OBJ_TRANSLATE || h->kind == RTR_OBJ_YROTATE) nchain++;
      else nprim++;
      if (h->kind == RTR_OBJ_BVH || h->kind == RTR_OBJ_GROUP) {
        int pass = h->kind == RTR_OBJ_GROUP || aabb_hit(&h->u.bvh.box, &ray, tmin, tmax);
        if (pass && (g_tf[cur] || (g_nprims[cur] >= g_dyn_min && !aabb_hit(&g_xfbox[cur], &ray, tmin, tmax)))) {
          macro++; mprims += g_nprims[cur]; sah += 2.0 * log2((double)g_nprims[cur] + 1) + 4; child_m = 1;
        }
      }
    }
#define PUSH(x) do { s->data[s->count] = (x); inm[s->count] = (uint8_t)child_m; s->count++; } while (0)
    switch (h->kind) {
      case RTR_OBJ_SPHERE: {
        const rtr_sphere *sp = &h->u.sphere;
        vec3 center = line_at(sp->center, ray.time, sp->motion);
        vec3 oc = sub(center, ray.origin);
        float a = dot(ray.direction, ray.direction);
        float b = -2.0f * dot(ray.direction, oc);
        float c = dot(oc, oc) - sp->radius * sp->radius;
        float disc = b * b - 4 * a * c;
        if (disc >= 0) {
          float sq = sqrtf(disc);
          float rt = (-b - sq) / (2.0f * a);
          if (tmin >= rt || rt >= tmax) rt = (-b + sq) / (2.0f * a);
          if (tmin < rt && rt < tmax) tmax = rt;
        }
      } break;
      case RTR_OBJ_BVH: {
        const rtr_bvh *n = &h->u.bvh;
        if (aabb_hit(&n->box, &ray, tmin, tmax)) { PUSH(sc->refs[n->right]); PUSH(sc->refs[n->left]); }
      } break;
      case RTR_OBJ_TRIANGLE: case RTR_OBJ_QUAD: {
        int tri = h->kind == RTR_OBJ_TRIANGLE;
        float al, be, t; vec3 p;
        plane_hit(&h->u.planar.geom, &ray, tmin, tmax, &al, &be, &t, &p);
        int inside = (0.0f <= al && al <= 1.0f) && (0.0f <= be && be <= 1.0f) && (!tri || al + be <= 1.0f);
        if (inside) tmax = t;
      } break;
      case RTR_OBJ_TRANSLATE: {
        const rtr_translate *tr = &h->u.translate;
        if (in_m) { fprintf(stderr, "chain entered inside a macro!\n"); abort(); }
        if (tc == 0) { ray.origin = sub(ray.origin, tr->offset); PUSH(cur); PUSH(tr->child); tc++; K++; }
        else { ray.origin = add(ray.origin, tr->offset); tc--; }
      } break;
      case RTR_OBJ_YROTATE: {
        const rtr_yrotate *y = &h->u.yrotate;
        float sn = y->sin_theta, cs = y->cos_theta;
        vec3 o = ray.origin, d = ray.direction;
        if (yc == 0) {
          ray.origin = v3((cs * o.x) - (sn * o.z), o.y, (sn * o.x) + (cs * o.z));
          ray.direction = v3((cs * d.x) - (sn * d.z), d.y, (sn * d.x) + (cs * d.z));
          PUSH(cur); PUSH(y->child); yc++;
        } else {
          ray.origin = v3((cs * o.x) + (sn * o.z), o.y, (-sn * o.x) + (cs * o.z));
          ray.direction = v3((cs * d.x) + (sn * d.z), d.y, (-sn * d.x) + (cs * d.z));
          yc--;
        }
      } break;
      case RTR_OBJ_GROUP:
        for (uint16_t i = 0; i < h->u.group.count; ++i) PUSH((uint16_t)(h->u.group.first + i));
        break;
    }
#undef PUSH
  }
  free(s);
  st[S_DBVH] += nbvh; st[S_DBVHPASS] += nbvhpass; st[S_DCHAIN] += nchain; st[S_DPRIM] += nprim; st[S_DGROUP] += ngroup;
  if (K == 0) { st[S_DTOP_K0] += top; st[S_DRAYS_K0] += 1; }
  st[S_DTOP] += top; st[S_DMACRO] += macro; st[S_DMPRIMS] += mprims; st[S_DSAH] += sah;
}

/* ray_color of the oracle with the analysis before every hit() */
static void trace_pixel(const rt_scene *sc, const rt_camera *cam, const rt_params *p, int32_t i, int32_t j,
                        href_stack *hs, counters *cn, double *st) {
  xw_state rng;
  xw_init(p->seed, (uint64_t)i * (uint64_t)p->width + (uint64_t)j, &rng);
  vec3 pixel_point = add(cam->pixel00, add(scale((float)i, cam->delta_v), scale((float)j, cam->delta_u)));
  for (int32_t sN = 0; sN < p->samples_per_pixel; ++sN) {
    ray_t ray;
    ray.origin = cam->center;
    float xo = uniform(&rng, cn) - 0.5f;
    float yo = uniform(&rng, cn) - 0.5f;
    ray.direction = sub(pixel_point, ray.origin);
    ray.direction = add(ray.direction, scale(xo, cam->delta_u));
    ray.direction = add(ray.direction, scale(yo, cam->delta_v));
    ray.time = uniform(&rng, cn);
    int32_t bounces = (int32_t)(uint8_t)p->max_bounces;
    hit_rec rec;
    memset(&rec, 0, sizeof rec);
    uint16_t root = sc->refs[sc->root];
    while (bounces > 0) {
      walk(sc, &ray, st);
      if (!hit(sc, hs, root, 0.001f, INFINITY, &ray, &rec, cn)) break;
      scatter_t sct = scatter(sc, &rng, &rec, ray.direction, cn);
      if (!sct.is_hit) break;
      ray.origin = rec.point;
      ray.direction = sct.direction;
      bounces--;
    }
  }
}

int xf_analyze(const rt_scene *sc, const rt_camera *cam, const rt_params *p, int pixel_stride, double *out, int dedup, int dyn_min) {
  g_dedup = dedup; g_dyn_min = (uint32_t)dyn_min;
  if (!g_jump_ready) xw_build_tables();
  g_tf = (uint8_t *)malloc(sc->hittable_count);
  g_xfpar = (uint8_t *)calloc(sc->hittable_count, 1);
  memset(g_tf, 2, sc->hittable_count);
  for (uint32_t r = 0; r < sc->hittable_count; ++r) tf_of(sc, (uint16_t)r);
  g_xfbox = (rtr_aabb *)malloc(sizeof(rtr_aabb) * sc->hittable_count);
  g_hasxf = (uint8_t *)malloc(sc->hittable_count);
  g_nprims = (uint32_t *)calloc(sc->hittable_count, 4);
  memset(g_hasxf, 2, sc->hittable_count);
  for (uint32_t r = 0; r < sc->hittable_count; ++r) xfbox_of(sc, (uint16_t)r);
  double tot[S_NSTAT] = {0};
  int64_t n = (int64_t)p->width * p->height;
#pragma omp parallel
  {
    double st[S_NSTAT] = {0};
    counters cn; memset(&cn, 0, sizeof cn);
    href_stack *hs = (href_stack *)malloc(sizeof(href_stack));
    hs->count = 0; hs->max_seen = 0; hs->overflow = 0;
#pragma omp for schedule(dynamic, 64)
    for (int64_t k = 0; k < n; k += pixel_stride)
      trace_pixel(sc, cam, p, (int32_t)(k / p->width), (int32_t)(k % p->width), hs, &cn, st);
#pragma omp critical
    for (int q = 0; q < S_NSTAT; ++q) tot[q] += st[q];
    free(hs);
  }
  for (int q = 0; q < S_NSTAT; ++q) out[q] = tot[q];
  int ntf = 0, nxp = 0;
  for (uint32_t r = 0; r < sc->hittable_count; ++r) { ntf += g_tf[r]; nxp += g_xfpar[r]; }
  out[S_NSTAT] = ntf; out[S_NSTAT + 1] = nxp;
  double mem = 0, ntop = 0;
  for (uint32_t r = 0; r < sc->hittable_count; ++r)
    if (!g_tf[r] && (sc->hittables[r].kind == RTR_OBJ_BVH || sc->hittables[r].kind == RTR_OBJ_GROUP) && g_nprims[r] >= g_dyn_min) { mem += g_nprims[r]; ntop++; }
  out[S_NSTAT + 2] = mem; out[S_NSTAT + 3] = ntop;
  free(g_tf); free(g_xfpar);
  return 0;
}
