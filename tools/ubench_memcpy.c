/* Host memcpy rate for the reader's Read() copies (16 MiB in 16 KiB pieces, and whole): calibration only. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec*1e3+t.tv_nsec/1e6;}
int main(){size_t n=16777216; char*a=malloc(n),*b=malloc(16384); memset(a,1,n);
double best=1e9; for(int r=0;r<10;r++){double t=now(); for(size_t o=0;o<n;o+=16384) memcpy(b,a+o,16384); double e=now()-t; if(e<best)best=e;}
printf("16MB in 16KB pieces into one 16KB buffer: %.3f ms (%.1f GB/s)\n",best,n/best/1e6);
char*c=malloc(n); memset(c,0,n); best=1e9; for(int r=0;r<10;r++){double t=now(); memcpy(c,a,n); double e=now()-t; if(e<best)best=e;}
printf("16MB memcpy to a fresh buffer: %.3f ms (%.1f GB/s)\n",best,n/best/1e6);return b[5]+c[7];}
