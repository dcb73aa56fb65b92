/* gen_tsp.c — TSP instance for e3_tsp: n cities, d[i][i+1] = 10, every other
 * distance uniform in [10, 1010) -> the path 0 -> 1 -> ... -> n-1 (length
 * 10 (n-1)) is planted.  Usage: gen_tsp [n] [seed] */
#include <stdio.h>
#include <stdlib.h>

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 100;
  srand(argc > 2 ? (unsigned)atoi(argv[2]) : 1u);
  printf("%d\n", n);
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < n; ++j) printf("%d ", j == i + 1 ? 10 : 10 + rand() % 1000);
    printf("\n");
  }
  return 0;
}
