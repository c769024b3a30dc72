/*
 * Deterministic synthetic orchard point-cloud generator.
 *
 * Produces a PointCloud2-shaped byte buffer (point_step 16: x, y, z, intensity as float32,
 * is_dense = true) plus the exploration polygon that the aos_seed_gen_node would receive on
 * /aos_planner/exploration_area (float32 Point32 vertices, widened to double like
 * src/aos_seed_gen_node.cpp:258-260 does).
 *
 * Reproducibility rules: every point owns an independent SplitMix64 stream seeded from
 * (seed, point index), so generation is order- and thread-count-independent; only + - * are
 * used on doubles (no libm transcendentals; discs by rejection sampling); build with
 * -ffp-contract=off so no FMA changes a rounding.
 *
 * Scene: square polygon [0, L]^2 with L = n_grid*res - 5 - res/2 (so the seed-gen grid is
 * exactly n_grid x n_grid, origin (-2.5, -2.5)); tree rows parallel to x, every 3.5 m from
 * y = 2; trees every 1.2 m from x = 2.  Points: 60 % canopy (disc r = 0.5 m around a tree;
 * z in [-0.3, 0.4] for 80 %, [0.6, 3.0] for 20 %), ground (z in [-1.3, -1.1]),
 * outlier_frac outliers (z in [-0.4, 0.5]), the rest ground.
 *
 * This is not product code and not the oracle: it only manufactures inputs.
 */
#include <stdint.h>
#include <string.h>

typedef struct orchard_cfg {
    uint64_t seed;
    uint64_t n_points;
    int32_t  grid_n;       /* grid cells per side (W = H = grid_n)            */
    float    res;          /* grid resolution (float, as the node stores it)  */
    int32_t  max_rows;     /* 0 = fill the square                             */
    double   row_x_end;    /* 0 = L - 2                                       */
    double   outlier_frac; /* fraction of isolated in-clip outliers (default 0.01; SURVEY said 0.10,
                              which is a uniform fog dense enough that ROR survivors bridge every
                              inter-row gap — see DESIGN.md "Synthetic input")               */
} orchard_cfg;

static inline uint64_t sm64_next(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline double u01(uint64_t *s) { return (double)(sm64_next(s) >> 11) * (1.0 / 9007199254740992.0); }
static inline double uab(uint64_t *s, double a, double b) { return a + (b - a) * u01(s); }

float orchard_side_length(int32_t grid_n, float res) {
    return (float)((double)grid_n * (double)res - 5.0 - (double)res / 2.0);
}

/* Rows / trees of the scene. Returns number of trees; fills up to cap centres (x, y). */
static int64_t orchard_trees(const orchard_cfg *c, double *cx, double *cy, int64_t cap) {
    const double L = (double)orchard_side_length(c->grid_n, c->res);
    const double x_end = c->row_x_end > 0.0 ? c->row_x_end : L - 2.0;
    int64_t n = 0;
    int32_t rows = 0;
    for (double y = 2.0; y <= L - 2.0; y += 3.5) {
        if (c->max_rows > 0 && rows >= c->max_rows) break;
        for (double x = 2.0; x <= x_end; x += 1.2) {
            if (n < cap) { cx[n] = x; cy[n] = y; }
            ++n;
        }
        ++rows;
    }
    return n;
}

int64_t orchard_num_trees(const orchard_cfg *c) { return orchard_trees(c, 0, 0, 0); }

/* Square polygon as 4 (x, y) doubles that came from float32 Point32. */
void orchard_polygon(const orchard_cfg *c, double *poly_xy /* 8 */) {
    const float L = orchard_side_length(c->grid_n, c->res);
    const float v[8] = {0.0f, 0.0f, L, 0.0f, L, L, 0.0f, L};
    for (int i = 0; i < 8; ++i) poly_xy[i] = (double)v[i];
}

/* Fills n_points * 16 bytes. tree_xy scratch: 2 * orchard_num_trees doubles. */
void orchard_generate_range(const orchard_cfg *c, const double *tree_x, const double *tree_y,
                            int64_t n_trees, uint64_t begin, uint64_t end, uint8_t *out) {
    const double L = (double)orchard_side_length(c->grid_n, c->res);
    for (uint64_t i = begin; i < end; ++i) {
        uint64_t s = c->seed * 0xD1B54A32D192ED03ULL ^ (i * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL);
        sm64_next(&s);
        const double kind = u01(&s);
        double x, y, z;
        if (kind < 0.6 && n_trees > 0) {
            int64_t t = (int64_t)(u01(&s) * (double)n_trees);
            if (t >= n_trees) t = n_trees - 1;
            double dx, dy;
            do { dx = uab(&s, -0.5, 0.5); dy = uab(&s, -0.5, 0.5); } while (dx * dx + dy * dy > 0.25);
            x = tree_x[t] + dx;
            y = tree_y[t] + dy;
            z = (u01(&s) < 0.8) ? uab(&s, -0.3, 0.4) : uab(&s, 0.6, 3.0);
        } else if (kind < 1.0 - c->outlier_frac) {
            x = uab(&s, 0.0, L); y = uab(&s, 0.0, L); z = uab(&s, -1.3, -1.1);
        } else {
            x = uab(&s, 0.0, L); y = uab(&s, 0.0, L); z = uab(&s, -0.4, 0.5);
        }
        float rec[4] = {(float)x, (float)y, (float)z, (float)(i & 0xFF)};
        memcpy(out + 16 * i, rec, 16);
    }
}

int64_t orchard_tree_centres(const orchard_cfg *c, double *tree_x, double *tree_y, int64_t cap) {
    return orchard_trees(c, tree_x, tree_y, cap);
}

/* One scan of the streaming config C4: points [begin, end) of scan `scan`, i.e. the
 * scene restricted to the disc of radius scan_r around the pose (px, py). Canopy points come from
 * the trees given (the caller passes those whose disc can reach the scan disc), ground and outliers
 * are uniform in the scan disc (rejection from its bounding square). Every point owns its own
 * SplitMix64 stream seeded from (seed, scan, index). */
void orchard_generate_scan(const orchard_cfg *c, const double *tree_x, const double *tree_y, int64_t n_trees,
                           uint64_t scan, double px, double py, double scan_r, uint64_t begin, uint64_t end,
                           uint8_t *out) {
    const double r2 = scan_r * scan_r;
    for (uint64_t i = begin; i < end; ++i) {
        uint64_t s = (c->seed * 0xD1B54A32D192ED03ULL) ^ (scan * 0xA24BAED4963EE407ULL) ^
                     (i * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL);
        sm64_next(&s);
        const double kind = u01(&s);
        double x = px, y = py, z;
        if (kind < 0.6 && n_trees > 0) {
            for (int tries = 0; tries < 64; ++tries) {
                int64_t t = (int64_t)(u01(&s) * (double)n_trees);
                if (t >= n_trees) t = n_trees - 1;
                double dx, dy;
                do { dx = uab(&s, -0.5, 0.5); dy = uab(&s, -0.5, 0.5); } while (dx * dx + dy * dy > 0.25);
                x = tree_x[t] + dx;
                y = tree_y[t] + dy;
                if ((x - px) * (x - px) + (y - py) * (y - py) <= r2) break;
            }
            z = (u01(&s) < 0.8) ? uab(&s, -0.3, 0.4) : uab(&s, 0.6, 3.0);
        } else {
            double dx, dy;
            do { dx = uab(&s, -scan_r, scan_r); dy = uab(&s, -scan_r, scan_r); } while (dx * dx + dy * dy > r2);
            x = px + dx;
            y = py + dy;
            z = (kind < 1.0 - c->outlier_frac) ? uab(&s, -1.3, -1.1) : uab(&s, -0.4, 0.5);
        }
        float rec[4] = {(float)x, (float)y, (float)z, (float)(i & 0xFF)};
        memcpy(out + 16 * i, rec, 16);
    }
}
