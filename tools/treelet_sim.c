/* Dev tool for tools/treelet_sim.py: subtree sizes of a BVH2 in DFS preorder
 * (node i's left child is i+1, its right child i+1+size(left)).
 * gcc -O2 -shared -fPIC -o tools/treelet_sim.so tools/treelet_sim.c */
#include <stdint.h>

/* size[i] = nodes in the subtree of i; prims[i] = leaf candidates in it;
 * right[i] = right child (-1 for leaves) */
void subtree_sizes(int64_t n, const int32_t* count, int64_t* size, int64_t* prims, int64_t* right) {
    for (int64_t i = n - 1; i >= 0; --i) {
        if (count[i] > 0) {
            size[i] = 1;
            prims[i] = count[i];
            right[i] = -1;
        } else {
            const int64_t l = i + 1, r = i + 1 + size[i + 1];
            size[i] = 1 + size[l] + size[r];
            prims[i] = prims[l] + prims[r];
            right[i] = r;
        }
    }
}
