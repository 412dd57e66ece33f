// main.cpp -- bin/meshclust (src/cluster/src/main.cpp:25-26 equivalent).
#include "runner.hpp"

int main(int argc, char **argv) { return mc::meshclust_main(argc, argv); }
