/* mjh_convex.h — general convex narrowphase: GJK + EPA, one contact per pair.
 *
 * MuJoCo routes every geom pair without a dedicated function (sphere-ellipsoid,
 * capsule-{ellipsoid,cylinder}, ellipsoid-{ellipsoid,cylinder,box},
 * cylinder-{cylinder,box}) to its convex collider (engine_collision_convex.c
 * mjc_Convex; since 3.3 the native GJK/EPA of engine_collision_gjk.c, one
 * contact unless mjENBL_MULTICCD); MuJoCo Warp does the same with its gjk/epa
 * in collision_gjk.py. This file restates that published algorithm:
 *
 *   geom1 is inflated by the pair margin (a Minkowski sum with a ball), so one
 *   intersection test covers "within margin"; GJK (Voronoi-region simplex
 *   descent) either finds a separating direction (no contact) or a
 *   tetrahedron of Minkowski-difference points w = a - b enclosing the
 *   origin; EPA grows that polytope towards the difference's boundary until
 *   the face nearest the origin is within CVX_TOL of the support along its
 *   normal. That face gives the penetration depth p (of the inflated pair),
 *   the normal n (from geom1 to geom2) and, by the barycentric coordinates of
 *   the origin's projection, witness points a (geom1) and b (geom2):
 *     dist = margin - p,  pos = ((a - margin n) + b) / 2,  frame normal = n.
 *
 * EPA converges linearly where both surfaces are curved (sphere, ellipsoid,
 * cylinder rims): each vertex refines one face, and its tolerance bounds the
 * depth's error but the normal's only by its square root. So the normal is
 * then polished by Newton's method on the overlap
 * f(u) = h1(u) + h2(-u) over unit u (h: support function; the penetration
 * depth is min f, the normal its minimiser): exact gradient (the support
 * point of the difference, projected on the tangent plane), Hessian by
 * central differences of it, steps only along positive-curvature
 * eigen-directions (a kink, where a flat side meets an edge, shows as a huge
 * curvature and gets no step), each step accepted only if f decreases. The
 * position then comes from the strictly convex geom's support point
 * (sphere/ellipsoid; otherwise the EPA witness).
 *
 * The same source is compiled into the HIP step (float32, csrc/mjh_step.hip
 * narrowphase) and the CPU oracle (float64/float32, oracle/oracle.c collide),
 * so oracle agreement checks precision only; the algorithm is pinned by
 * closed-form and support-function known answers (tests/test_convex.py).
 * Includers define CVX_REAL (C) or compile as HIP (float). Computation runs
 * in geom1-centred coordinates so float32 keeps the shapes' resolution away
 * from the world origin.
 */
#ifndef MJH_CONVEX_H
#define MJH_CONVEX_H

#if defined(__HIPCC__)
typedef float cvx_real;
#define CVX_FN static __device__ inline
#define CVX_ENTRY static __device__ __noinline__
#define CVX_SQRT sqrtf
#define CVX_FABS fabsf
#else
typedef CVX_REAL cvx_real;
#define CVX_FN static inline
#define CVX_ENTRY static
#define CVX_SQRT sqrt
#define CVX_FABS fabs
#endif

#define CVX_GJK_ITERS 40 /* simplex descents before giving up (no contact) */
#define CVX_NV 32        /* EPA polytope vertices (the iteration cap is CVX_NV - 4) */
#define CVX_NF 64        /* EPA polytope faces */
#define CVX_NE 32        /* EPA horizon edges per expansion */
#define CVX_TOL ((cvx_real)1e-6) /* EPA convergence: support gap along the nearest face's normal (m) */
#define CVX_POLISH_ITERS 6         /* Newton polish iterations after an unconverged EPA */
#define CVX_POLISH_FD ((cvx_real)1e-4) /* central-difference step for the polish's Hessian (rad) */
#define CVX_KINK ((cvx_real)50)        /* curvature above this x the size scale: a kink, no step */
#define CVX_KINK_BISECT 30             /* bisection steps locating a kink (of a 4e-4 rad bracket) */
#define CVX_LINE_EPS ((cvx_real)1e-12) /* squared: origin this close to a simplex edge's line is on it */
#define CVX_FACE_EPS ((cvx_real)1e-10) /* sine below which a triangle counts as degenerate */

/* geom types: 2 sphere, 3 capsule, 4 ellipsoid, 5 cylinder, 6 box (MuJoCo mjtGeom) */
typedef struct {
  int type;
  cvx_real pos[3], mat[9], size[3]; /* mat row-major, column k = local axis k */
  cvx_real infl;                    /* margin added all round (geom1 only) */
} cvx_geom;

typedef struct {
  cvx_real w[3], a[3]; /* Minkowski-difference point w = a - b; a on geom1 */
} cvx_vert;

typedef struct {
  signed char v[3];   /* vertex indices, counter-clockwise seen from outside; v[0] < 0: free slot */
  signed char adj[3]; /* adj[q]: the face across the edge v[q] -> v[q + 1] */
  cvx_real n[3], d;   /* outward unit normal, distance of the plane from the origin */
} cvx_face;

CVX_FN cvx_real cvx_dot(const cvx_real* a, const cvx_real* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
CVX_FN void cvx_cross(cvx_real* r, const cvx_real* a, const cvx_real* b) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
CVX_FN void cvx_sub(cvx_real* r, const cvx_real* a, const cvx_real* b) {
  r[0] = a[0] - b[0];
  r[1] = a[1] - b[1];
  r[2] = a[2] - b[2];
}
CVX_FN void cvx_copy(cvx_real* r, const cvx_real* a) {
  r[0] = a[0];
  r[1] = a[1];
  r[2] = a[2];
}
/* (a x b) x a: the component of b perpendicular to a (times |a|^2) */
CVX_FN void cvx_perp_toward(cvx_real* r, const cvx_real* a, const cvx_real* b) {
  cvx_real t[3];
  cvx_cross(t, a, b);
  cvx_cross(r, t, a);
}
/* some vector perpendicular to a: a x (the axis a is least aligned with) */
CVX_FN void cvx_any_perp(cvx_real* r, const cvx_real* a) {
  cvx_real e[3] = {0, 0, 0};
  const cvx_real x = CVX_FABS(a[0]), y = CVX_FABS(a[1]), z = CVX_FABS(a[2]);
  e[x <= y && x <= z ? 0 : (y <= z ? 1 : 2)] = 1;
  cvx_cross(r, a, e);
}

/* support point of g in direction d (world-aligned, geom1-centred coordinates) */
CVX_FN void cvx_support(const cvx_geom* g, const cvx_real* d, cvx_real* out) {
  const cvx_real* m = g->mat;
  const cvx_real* s = g->size;
  cvx_real l[3], p[3] = {0, 0, 0}, rad = g->infl;
  for (int k = 0; k < 3; k++) l[k] = m[k] * d[0] + m[3 + k] * d[1] + m[6 + k] * d[2];
  switch (g->type) {
    case 2: /* sphere: the centre plus the radius along d */
      rad += s[0];
      break;
    case 3: /* capsule: the segment end along d plus the radius */
      p[2] = l[2] >= 0 ? s[1] : -s[1];
      rad += s[0];
      break;
    case 4: { /* ellipsoid: S^2 l / |S l| */
      const cvx_real u[3] = {s[0] * l[0], s[1] * l[1], s[2] * l[2]};
      const cvx_real un = CVX_SQRT(cvx_dot(u, u));
      if (un > 0)
        for (int k = 0; k < 3; k++) p[k] = s[k] * u[k] / un;
      break;
    }
    case 5: { /* cylinder: the rim point along d's radial part, the cap along d's axial part */
      const cvx_real rl = CVX_SQRT(l[0] * l[0] + l[1] * l[1]);
      if (rl > 0) {
        p[0] = s[0] * l[0] / rl;
        p[1] = s[0] * l[1] / rl;
      }
      p[2] = l[2] >= 0 ? s[1] : -s[1];
      break;
    }
    default: /* box: the corner along d */
      for (int k = 0; k < 3; k++) p[k] = l[k] >= 0 ? s[k] : -s[k];
      break;
  }
  const cvx_real dn = CVX_SQRT(cvx_dot(d, d));
  const cvx_real f = dn > 0 ? rad / dn : 0;
  for (int k = 0; k < 3; k++) out[k] = g->pos[k] + m[3 * k] * p[0] + m[3 * k + 1] * p[1] + m[3 * k + 2] * p[2] + f * d[k];
}

/* the Minkowski-difference vertex along d: a = s1(d), b = s2(-d), w = a - b */
CVX_FN void cvx_vertex(const cvx_geom* g1, const cvx_geom* g2, const cvx_real* d, cvx_vert* v) {
  cvx_real nd[3] = {-d[0], -d[1], -d[2]}, b[3];
  cvx_support(g1, d, v->a);
  cvx_support(g2, nd, b);
  cvx_sub(v->w, v->a, b);
}

/* the line case of the simplex descent: s[1] newest (A), s[0] (B) */
CVX_FN void cvx_line(cvx_vert* s, int* n, cvx_real* d) {
  cvx_real ab[3], ao[3] = {-s[1].w[0], -s[1].w[1], -s[1].w[2]};
  cvx_sub(ab, s[0].w, s[1].w);
  if (cvx_dot(ab, ao) > 0) {
    *n = 2;
    cvx_perp_toward(d, ab, ao);
    if (cvx_dot(d, d) <= CVX_LINE_EPS * cvx_dot(ab, ab) * cvx_dot(ab, ab)) cvx_any_perp(d, ab); /* origin on the line */
  } else {
    s[0] = s[1];
    *n = 1;
    cvx_copy(d, ao);
  }
}

/* the triangle case: s[2] newest (A), s[1] (B), s[0] (C) */
CVX_FN void cvx_triangle(cvx_vert* s, int* n, cvx_real* d) {
  cvx_real ab[3], ac[3], abc[3], t[3], ao[3] = {-s[2].w[0], -s[2].w[1], -s[2].w[2]};
  cvx_sub(ab, s[1].w, s[2].w);
  cvx_sub(ac, s[0].w, s[2].w);
  cvx_cross(abc, ab, ac);
  if (cvx_dot(abc, abc) <= CVX_FACE_EPS * CVX_FACE_EPS * cvx_dot(ab, ab) * cvx_dot(ac, ac)) { /* collinear: the edge A-B */
    s[0] = s[1];
    s[1] = s[2];
    cvx_line(s, n, d);
    return;
  }
  cvx_cross(t, abc, ac);
  if (cvx_dot(t, ao) > 0) {
    if (cvx_dot(ac, ao) > 0) { /* the edge A-C */
      s[1] = s[2];
      cvx_line(s, n, d);
      return;
    }
    s[0] = s[1];
    s[1] = s[2];
    cvx_line(s, n, d);
    return;
  }
  cvx_cross(t, ab, abc);
  if (cvx_dot(t, ao) > 0) { /* the edge A-B */
    s[0] = s[1];
    s[1] = s[2];
    cvx_line(s, n, d);
    return;
  }
  *n = 3;
  if (cvx_dot(abc, ao) >= 0) {
    cvx_copy(d, abc);
  } else { /* below the triangle: swap B and C so that d = the normal of C, B, A */
    const cvx_vert tmp = s[0];
    s[0] = s[1];
    s[1] = tmp;
    for (int k = 0; k < 3; k++) d[k] = -abc[k];
  }
}

/* the tetrahedron case: s[3] newest (A); 1 when the origin is enclosed */
CVX_FN int cvx_tetra(cvx_vert* s, int* n, cvx_real* d) {
  /* the three faces through A: (A, X, Y) with the opposite vertex Z */
  const int fx[3] = {2, 1, 0}, fy[3] = {1, 0, 2}, fz[3] = {0, 2, 1};
  cvx_real ao[3] = {-s[3].w[0], -s[3].w[1], -s[3].w[2]};
  for (int f = 0; f < 3; f++) {
    cvx_real ax[3], ay[3], az[3], nrm[3];
    cvx_sub(ax, s[fx[f]].w, s[3].w);
    cvx_sub(ay, s[fy[f]].w, s[3].w);
    cvx_sub(az, s[fz[f]].w, s[3].w);
    cvx_cross(nrm, ax, ay);
    if (cvx_dot(nrm, az) > 0)
      for (int k = 0; k < 3; k++) nrm[k] = -nrm[k];
    if (cvx_dot(nrm, ao) > 0) { /* the origin is beyond this face: descend to it */
      const cvx_vert x = s[fx[f]], y = s[fy[f]], a = s[3];
      s[0] = y;
      s[1] = x;
      s[2] = a;
      cvx_triangle(s, n, d);
      return 0;
    }
  }
  return 1;
}

/* GJK: 1 with s[0..3] a tetrahedron enclosing the origin (the pair
   intersects), 0 when a separating direction is found or the descent stalls */
CVX_FN int cvx_gjk(const cvx_geom* g1, const cvx_geom* g2, cvx_vert* s) {
  cvx_real d[3];
  cvx_sub(d, g2->pos, g1->pos);
  if (cvx_dot(d, d) <= 0) {
    d[0] = 1;
    d[1] = d[2] = 0;
  }
  int n = 0;
  for (int it = 0; it < CVX_GJK_ITERS; it++) {
    cvx_vert v;
    cvx_vertex(g1, g2, d, &v);
    if (cvx_dot(v.w, d) <= 0) return 0; /* the difference does not reach the origin along d */
    s[n++] = v;
    if (n == 1) {
      for (int k = 0; k < 3; k++) d[k] = -v.w[k];
      if (cvx_dot(d, d) <= 0) d[0] = 1; /* touching at one point: any direction */
      continue;
    }
    if (n == 2) cvx_line(s, &n, d);
    else if (n == 3) cvx_triangle(s, &n, d);
    else if (cvx_tetra(s, &n, d)) return 1;
    if (cvx_dot(d, d) <= 0) return 0;
  }
  return 0;
}

/* a face through vertices i, j, k (counter-clockwise from outside); 0 if degenerate */
CVX_FN int cvx_face_make(cvx_face* f, const cvx_vert* v, int i, int j, int k) {
  cvx_real e1[3], e2[3], nrm[3];
  cvx_sub(e1, v[j].w, v[i].w);
  cvx_sub(e2, v[k].w, v[i].w);
  cvx_cross(nrm, e1, e2);
  const cvx_real nl = CVX_SQRT(cvx_dot(nrm, nrm));
  if (!(nl > CVX_FACE_EPS * CVX_SQRT(cvx_dot(e1, e1) * cvx_dot(e2, e2)))) return 0;
  for (int q = 0; q < 3; q++) f->n[q] = nrm[q] / nl;
  f->d = cvx_dot(f->n, v[i].w);
  f->v[0] = (signed char)i;
  f->v[1] = (signed char)j;
  f->v[2] = (signed char)k;
  return 1;
}

/* a length scale of g: an upper bound on its radii of curvature is a few of these */
CVX_FN cvx_real cvx_scale(const cvx_geom* g) {
  const cvx_real* s = g->size;
  switch (g->type) {
    case 2: return s[0];
    case 3: case 5: return s[0] + s[1];
    default: return s[0] + s[1] + s[2];
  }
}

/* f(u) = h1(u) + h2(-u) for unit u, with the difference's support vertex */
CVX_FN cvx_real cvx_overlap(const cvx_geom* g1, const cvx_geom* g2, const cvx_real* u, cvx_vert* v) {
  cvx_vertex(g1, g2, u, v);
  return cvx_dot(v->w, u);
}

/* Newton polish of the unit normal u (see the header comment); *depth =
   f(u) at the end, *v its support vertex; 1 if any step was accepted */
CVX_FN int cvx_polish(const cvx_geom* g1, const cvx_geom* g2, cvx_real* u, cvx_real* depth, cvx_vert* v) {
  cvx_real f = cvx_overlap(g1, g2, u, v);
  const cvx_real kink = CVX_KINK * (cvx_scale(g1) + cvx_scale(g2) + g1->infl);
  int improved = 0, nk = 0;
  cvx_real kdir[3] = {0, 0, 0}; /* the last iteration's kink direction (nk == 1) */
  for (int it = 0; it < CVX_POLISH_ITERS; it++) {
    cvx_real t[2][3], dw[2][3], g[2];
    cvx_any_perp(t[0], u);
    const cvx_real tl = CVX_SQRT(cvx_dot(t[0], t[0]));
    for (int k = 0; k < 3; k++) t[0][k] /= tl;
    cvx_cross(t[1], u, t[0]);
    for (int j = 0; j < 2; j++) {
      cvx_real up[3], um[3];
      cvx_vert vp, vm;
      for (int k = 0; k < 3; k++) {
        up[k] = u[k] + CVX_POLISH_FD * t[j][k];
        um[k] = u[k] - CVX_POLISH_FD * t[j][k];
      }
      cvx_vertex(g1, g2, up, &vp);
      cvx_vertex(g1, g2, um, &vm);
      for (int k = 0; k < 3; k++) dw[j][k] = (vp.w[k] - vm.w[k]) / (2 * CVX_POLISH_FD);
      g[j] = cvx_dot(v->w, t[j]);
    }
    /* the tangent-plane Hessian of f: t_i (d^2 h) t_j - f delta_ij, and its eigen-directions */
    const cvx_real h00 = cvx_dot(dw[0], t[0]) - f, h11 = cvx_dot(dw[1], t[1]) - f;
    const cvx_real h01 = (cvx_real)0.5 * (cvx_dot(dw[0], t[1]) + cvx_dot(dw[1], t[0]));
    const cvx_real mean = (cvx_real)0.5 * (h00 + h11), hd = (cvx_real)0.5 * (h00 - h11);
    const cvx_real rad = CVX_SQRT(hd * hd + h01 * h01);
    cvx_real e[2] = {1, 0};
    if (rad > 0) { /* the eigenvector of mean + rad: (hd + rad, h01) or, if that vanishes, (h01, rad - hd) */
      if (hd >= 0) {
        e[0] = hd + rad;
        e[1] = h01;
      } else {
        e[0] = h01;
        e[1] = rad - hd;
      }
      const cvx_real el = CVX_SQRT(e[0] * e[0] + e[1] * e[1]);
      e[0] /= el;
      e[1] /= el;
    }
    const cvx_real lam[2] = {mean + rad, mean - rad}, ev[2][2] = {{e[0], e[1]}, {-e[1], e[0]}};
    cvx_real x[2] = {0, 0};
    nk = 0;
    for (int i = 0; i < 2; i++) {
      if (lam[i] > kink) { /* a kink: no Newton step across it */
        nk++;
        for (int k = 0; k < 3; k++) kdir[k] = ev[i][0] * t[0][k] + ev[i][1] * t[1][k];
        continue;
      }
      if (!(lam[i] > 0)) continue; /* no curvature (flat, saddle): no step */
      const cvx_real c = (g[0] * ev[i][0] + g[1] * ev[i][1]) / lam[i];
      x[0] -= c * ev[i][0];
      x[1] -= c * ev[i][1];
    }
    const cvx_real xl = CVX_SQRT(x[0] * x[0] + x[1] * x[1]);
    if (xl > (cvx_real)0.2) { /* at most 0.2 rad per step */
      x[0] *= (cvx_real)0.2 / xl;
      x[1] *= (cvx_real)0.2 / xl;
    }
    int accepted = 0;
    for (int bt = 0; bt < 4 && !accepted; bt++, x[0] *= (cvx_real)0.5, x[1] *= (cvx_real)0.5) {
      cvx_real un[3];
      for (int k = 0; k < 3; k++) un[k] = u[k] + x[0] * t[0][k] + x[1] * t[1][k];
      const cvx_real ul = CVX_SQRT(cvx_dot(un, un));
      for (int k = 0; k < 3; k++) un[k] /= ul;
      cvx_vert vn;
      const cvx_real fn = cvx_overlap(g1, g2, un, &vn);
      if (fn < f) {
        f = fn;
        *v = vn;
        cvx_copy(u, un);
        accepted = 1;
      }
    }
    if (!accepted) break;
    improved = 1;
    if (x[0] * x[0] + x[1] * x[1] < (cvx_real)1e-14) break;
  }
  if (nk == 1) {
    /* f is V-shaped across one kink, which lies within the difference
       stencil: bisect on the sign of f's slope along kdir */
    cvx_real lo = -2 * CVX_POLISH_FD, hi = 2 * CVX_POLISH_FD, un[3];
    cvx_vert vn;
    for (int it = 0; it < 2 + CVX_KINK_BISECT; it++) {
      const cvx_real tau = it == 0 ? lo : (it == 1 ? hi : (cvx_real)0.5 * (lo + hi));
      for (int k = 0; k < 3; k++) un[k] = u[k] + tau * kdir[k];
      const cvx_real ul = CVX_SQRT(cvx_dot(un, un));
      for (int k = 0; k < 3; k++) un[k] /= ul;
      cvx_vertex(g1, g2, un, &vn);
      const cvx_real kd = cvx_dot(kdir, un), slope = cvx_dot(vn.w, kdir) - kd * cvx_dot(vn.w, un);
      if (it == 0 && !(slope < 0)) break; /* not a V within the bracket */
      if (it == 1 && !(slope > 0)) break;
      if (it >= 2) {
        if (slope > 0) hi = tau;
        else lo = tau;
      }
    }
    const cvx_real tau = (cvx_real)0.5 * (lo + hi);
    for (int k = 0; k < 3; k++) un[k] = u[k] + tau * kdir[k];
    const cvx_real ul = CVX_SQRT(cvx_dot(un, un));
    for (int k = 0; k < 3; k++) un[k] /= ul;
    const cvx_real fn = cvx_overlap(g1, g2, un, &vn);
    if (fn < f) {
      f = fn;
      *v = vn;
      cvx_copy(u, un);
      improved = 1;
    }
  }
  *depth = f;
  return improved;
}

/* Narrowphase entry: 1 contact (dist, pos, normal from geom1 to geom2) or 0.
   Types as MuJoCo's; p/m/s: world centre, rotation (row-major), size. */
CVX_ENTRY int cvx_collide(int t1, const cvx_real* p1, const cvx_real* m1, const cvx_real* s1, int t2,
                          const cvx_real* p2, const cvx_real* m2, const cvx_real* s2, cvx_real margin,
                          cvx_real* dist, cvx_real* pos, cvx_real* nrm) {
  cvx_geom g1, g2;
  g1.type = t1;
  g2.type = t2;
  for (int k = 0; k < 3; k++) {
    g1.pos[k] = 0;
    g2.pos[k] = p2[k] - p1[k];
    g1.size[k] = s1[k];
    g2.size[k] = s2[k];
  }
  for (int k = 0; k < 9; k++) {
    g1.mat[k] = m1[k];
    g2.mat[k] = m2[k];
  }
  g1.infl = margin;
  g2.infl = 0;

  cvx_vert v[CVX_NV];
  if (!cvx_gjk(&g1, &g2, v)) return 0;

  /* EPA: the enclosing tetrahedron, oriented so that face (0, 1, 2) faces
     away from vertex 3 (vertices 1 and 2 swapped otherwise); its four faces
     then wind consistently outwards, and each edge links its two faces */
  {
    cvx_real e1[3], e2[3], e3[3], c[3];
    cvx_sub(e1, v[1].w, v[0].w);
    cvx_sub(e2, v[2].w, v[0].w);
    cvx_sub(e3, v[3].w, v[0].w);
    cvx_cross(c, e1, e2);
    if (cvx_dot(c, e3) > 0) {
      const cvx_vert t = v[1];
      v[1] = v[2];
      v[2] = t;
    }
  }
  cvx_face f[CVX_NF];
  for (int i = 0; i < CVX_NF; i++) {
    f[i].v[0] = -1;
    f[i].adj[0] = f[i].adj[1] = f[i].adj[2] = 0; /* every link stays a valid face index */
  }
  {
    const int tri[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {1, 3, 2}};
    for (int i = 0; i < 4; i++)
      if (!cvx_face_make(&f[i], v, tri[i][0], tri[i][1], tri[i][2])) return 0; /* a flat simplex */
    for (int i = 0; i < 4; i++)
      for (int q = 0; q < 3; q++) {
        const int a = f[i].v[q], b = f[i].v[(q + 1) % 3];
        for (int j = 0; j < 4; j++)
          for (int r = 0; r < 3; r++)
            if (f[j].v[r] == b && f[j].v[(r + 1) % 3] == a) f[i].adj[q] = (signed char)j;
      }
  }
  cvx_face fb = f[0]; /* the nearest face of the last closed polytope */
  int nv = 4, converged = 0;
  for (;;) {
    int best = -1;
    for (int i = 0; i < CVX_NF; i++)
      if (f[i].v[0] >= 0 && (best < 0 || f[i].d < f[best].d)) best = i;
    fb = f[best];
    cvx_vert w;
    cvx_vertex(&g1, &g2, fb.n, &w);
    converged = cvx_dot(w.w, fb.n) - fb.d < CVX_TOL;
    if (converged || nv == CVX_NV) break;
    /* the faces the new vertex sees, grown from the nearest across edges (a
       connected region, so float noise elsewhere cannot tear the polytope);
       the edges to the faces it does not see form the horizon */
    signed char state[CVX_NF], stack[CVX_NF], he[CVX_NE][3];
    for (int i = 0; i < CVX_NF; i++) state[i] = 0; /* 0 untested, 1 seen, 2 not seen */
    int sp = 0, ne = 0, ok = 1, nfree = 0;
    state[best] = 1;
    stack[sp++] = (signed char)best;
    while (sp > 0 && ok) {
      const int fi = stack[--sp];
      for (int q = 0; q < 3 && ok; q++) {
        const int nb = f[fi].adj[q];
        if (nb < 0 || nb >= CVX_NF || f[nb].v[0] < 0) { /* a dangling link: the polytope is torn */
          ok = 0;
          break;
        }
        if (state[nb] == 0) {
          if (cvx_dot(f[nb].n, w.w) - f[nb].d > 0) {
            state[nb] = 1;
            stack[sp++] = (signed char)nb;
            continue;
          }
          state[nb] = 2;
        }
        if (state[nb] == 1) continue;
        if (ne == CVX_NE) {
          ok = 0;
          break;
        }
        he[ne][0] = f[fi].v[q];
        he[ne][1] = f[fi].v[(q + 1) % 3];
        he[ne][2] = (signed char)nb;
        ne++;
      }
    }
    for (int i = 0; i < CVX_NF; i++) nfree += f[i].v[0] < 0 || state[i] == 1;
    if (!ok || nfree < ne) break; /* out of room: keep the nearest face found */
    /* replace the seen faces by a fan from the new vertex over the horizon */
    for (int i = 0; i < CVX_NF; i++)
      if (state[i] == 1) f[i].v[0] = -1;
    v[nv] = w;
    signed char nf[CVX_NE];
    for (int t = 0, slot = 0; t < ne && ok; t++) {
      while (f[slot].v[0] >= 0) slot++;
      nf[t] = (signed char)slot;
      if (!cvx_face_make(&f[slot], v, he[t][0], he[t][1], nv)) ok = 0; /* degenerate: torn */
      const int nb = he[t][2];
      f[slot].adj[0] = (signed char)nb;
      f[slot].adj[1] = f[slot].adj[2] = -1; /* linked below; -1 if the horizon is not a simple loop */
      for (int r = 0; r < 3; r++)
        if (f[nb].v[r] == he[t][1] && f[nb].v[(r + 1) % 3] == he[t][0]) f[nb].adj[r] = (signed char)slot;
    }
    if (!ok) break; /* fb and the vertices it names are intact */
    for (int t = 0; t < ne; t++)
      for (int u2 = 0; u2 < ne; u2++)
        if (he[u2][0] == he[t][1]) { /* edge (b, new) of fan face t = edge (new, a) of fan face u2, reversed */
          f[nf[t]].adj[1] = nf[u2];
          f[nf[u2]].adj[2] = nf[t];
        }
    for (int t = 0; t < ne; t++)
      if (f[nf[t]].adj[1] < 0 || f[nf[t]].adj[2] < 0) ok = 0;
    nv++;
    if (!ok) break; /* a pinched horizon: keep the nearest face of the last closed polytope */
  }

  /* the origin's projection onto the nearest face, in barycentric coordinates */
  const cvx_real* w0 = v[fb.v[0]].w;
  cvx_real e1[3], e2[3], pr[3], q[3];
  cvx_sub(e1, v[fb.v[1]].w, w0);
  cvx_sub(e2, v[fb.v[2]].w, w0);
  for (int k = 0; k < 3; k++) pr[k] = fb.n[k] * fb.d;
  cvx_sub(q, pr, w0);
  const cvx_real d00 = cvx_dot(e1, e1), d01 = cvx_dot(e1, e2), d11 = cvx_dot(e2, e2);
  const cvx_real d20 = cvx_dot(q, e1), d21 = cvx_dot(q, e2), den = d00 * d11 - d01 * d01;
  cvx_real l1 = 0, l2 = 0;
  if (den > 0) {
    l1 = (d11 * d20 - d01 * d21) / den;
    l2 = (d00 * d21 - d01 * d20) / den;
  }
  const cvx_real l0 = 1 - l1 - l2;
  *dist = margin - fb.d;
  for (int k = 0; k < 3; k++) {
    const cvx_real a = l0 * v[fb.v[0]].a[k] + l1 * v[fb.v[1]].a[k] + l2 * v[fb.v[2]].a[k];
    const cvx_real b = a - pr[k]; /* sum l_i b_i = sum l_i (a_i - w_i) */
    nrm[k] = fb.n[k];
    pos[k] = p1[k] + (cvx_real)0.5 * (a - margin * fb.n[k] + b);
  }
  /* polish the normal and the depth (EPA's tolerance bounds the depth's
     error, but the normal's only by its square root where f is curved) */
  cvx_real u[3], depth;
  cvx_vert vs;
  cvx_copy(u, fb.n);
  int have_vs = 0;
  if (cvx_polish(&g1, &g2, u, &depth, &vs)) {
    have_vs = 1;
    *dist = margin - depth;
    cvx_copy(nrm, u);
  }
  /* a strictly convex geom (sphere, ellipsoid) has a unique support point
     along the normal: the contact is pinned to it (the EPA witness is a
     blend of support points around it) */
  const int sc1 = t1 == 2 || t1 == 4, sc2 = t2 == 2 || t2 == 4;
  if (!sc1 && !sc2) return 1;
  if (!have_vs) cvx_vertex(&g1, &g2, u, &vs);
  for (int k = 0; k < 3; k++) {
    if (sc1) /* geom1's surface point, then half the distance along the normal */
      pos[k] = p1[k] + vs.a[k] - margin * u[k] + (cvx_real)0.5 * (*dist) * u[k];
    else if (sc2) /* geom2's: b = a - w */
      pos[k] = p1[k] + vs.a[k] - vs.w[k] - (cvx_real)0.5 * (*dist) * u[k];
  }
  return 1;
}

#endif /* MJH_CONVEX_H */
