/* CPU emulation of the certified tolerance triangulation (csrc/triangulate.hip
 * undistort_pair_tol / normal_eq_null_vector / null_vector_delta2) against the oracle's exact
 * path: counts points whose f32 outputs would differ (must all be caught) and the fallback rate.
 * Build: gcc -O2 -ffp-contract=off tools/tri_cert_emu.c -o /tmp/tri_cert_emu -lm
 * Input: python tools/tri_cert_sets.py (writes /tmp/tri/sets.bin).  Usage: tri_cert_emu [NF32] */
#include "../oracle/cv_calib3d.c"
#include <stdio.h>
#include <stdlib.h>
/* ---------- proposed tolerance path (CPU emulation of the device arithmetic) ---------- */
static double dist_to_mid(double c){ /* |c - nearest f32 rounding midpoint| (same binade) */
  uint64_t b; memcpy(&b,&c,8); int64_t low = (int64_t)(b & 0x1FFFFFFFull); int E=(int)((b>>52)&0x7ff);
  double d = (double)llabs(low - (1<<28)); return ldexp(d, E-1075); }
static int NF32 = 3; static double KAP=8, C1=8, C2=0.1;
typedef struct { double ox, oy, delta; } UD;
static UD undist_tol(float uf, float vf, const double* c){
  const double cx=c[2], cy=c[5], ifx=1./c[0], ify=1./c[4];
  const double k1=c[9],k2=c[10],p1=c[11],p2=c[12],k3=c[13];
  double x0=((double)uf-cx)*ifx, y0=((double)vf-cy)*ify;
  float X0=(float)x0, Y0=(float)y0, cxx=0.f, cyy=0.f; float fk1=k1,fk2=k2,fk3=k3,fp1=p1,fp2=p2;
  float r2f=0, icf=1, xf=X0, yf=Y0; int neg=0;
  for(int j=0;j<NF32;j++){ xf=X0+cxx; yf=Y0+cyy; r2f=fmaf(xf,xf,yf*yf);
     float poly=r2f*fmaf(r2f,fmaf(r2f,fk3,fk2),fk1); icf=1.f/(1.f+poly); if(icf<0)neg=1;
     float xy=xf*yf; float dX=fmaf(2*fp1,xy,fp2*fmaf(2*xf,xf,r2f)); float dY=fmaf(fp1,fmaf(2*yf,yf,r2f),2*fp2*xy);
     cxx=-fmaf(X0,poly,dX)*icf; cyy=-fmaf(Y0,poly,dY)*icf; }
  /* Lipschitz bound at the last f32 iterate */
  float L = icf*(2*r2f*(fabsf(fk1)+r2f*(2*fabsf(fk2)+3*fabsf(fk3)*r2f)) + 8*(fabsf(fp1)+fabsf(fp2))*(fabsf(xf)+fabsf(yf)));
  double xd=x0+(double)cxx, yd=y0+(double)cyy;
  float polyl = r2f*fmaf(r2f,fmaf(r2f,fk3,fk2),fk1); float xyl=xf*yf;
  float dXl=fmaf(2*fp1,xyl,fp2*fmaf(2*xf,xf,r2f)), dYl=fmaf(fp1,fmaf(2*yf,yf,r2f),2*fp2*xyl);
  float e3 = KAP*5.96e-8f*((fabsf(X0)+fabsf(Y0))*fabsf(polyl)+fabsf(dXl)+fabsf(dYl))*icf;
  double e = e3;
  for(int j=NF32;j<5;j++){ double r2=fma(xd,xd,yd*yd); double ic=1/(1+((k3*r2+k2)*r2+k1)*r2); if(ic<0)neg=1;
     double dX=2*p1*xd*yd+p2*(r2+2*xd*xd), dY=p1*(r2+2*yd*yd)+2*p2*xd*yd; xd=(x0-dX)*ic; yd=(y0-dY)*ic; e*=L; }
  UD r; if(neg){xd=x0;yd=y0;}
  r.ox=fma(c[0],xd,fma(c[1],yd,c[2])); r.oy=fma(c[3],xd,fma(c[4],yd,c[5]));
  double ww=1/(c[6]*xd+c[7]*yd+c[8]); r.ox*=ww; r.oy*=ww;
  double kn = fabs(c[0])+fabs(c[1])+fabs(c[4]);
  r.delta = kn*(e + ldexp(fabs(xd)+fabs(yd),-46)) + ldexp(fabs(r.ox)+fabs(r.oy)+fabs(c[2])+fabs(c[5]),-45);  /* pixels */
  if (neg) r.delta = 1e300;
  return r; }
static int null_tol(double A[4][4], double nv[4], double* delta){
 double m[4][4]; for(int i=0;i<4;i++)for(int j=0;j<=i;j++){double s=A[0][i]*A[0][j]; for(int r=1;r<4;r++)s=fma(A[r][i],A[r][j],s); m[i][j]=s;}
 double D0=m[0][0],r0=1/D0; double l10=m[1][0]*r0,l20=m[2][0]*r0,l30=m[3][0]*r0;
 double a11=fma(-l10,m[1][0],m[1][1]),a21=fma(-l20,m[1][0],m[2][1]),a31=fma(-l30,m[1][0],m[3][1]);
 double a22=fma(-l20,m[2][0],m[2][2]),a32=fma(-l30,m[2][0],m[3][2]),a33=fma(-l30,m[3][0],m[3][3]);
 double r1=1/a11,l21=a21*r1,l31=a31*r1; double b22=fma(-l21,a21,a22),b32=fma(-l31,a21,a32),b33=fma(-l31,a31,a33);
 double r2=1/b22,l32=b32*r2; double D3=fma(-l32,b32,b33); if(!(fabs(D3)>=1e-30*D0))D3=1e-30*D0; double r3=1/D3;
 double x[4]; x[3]=r3; x[2]=-l32*x[3]; x[1]=-l21*x[2]-l31*x[3]; x[0]=-l10*x[1]-l20*x[2]-l30*x[3];
 double is=1/sqrt(x[0]*x[0]+x[1]*x[1]+x[2]*x[2]+x[3]*x[3]); for(int q=0;q<4;q++)x[q]*=is;
 double prev=1, dd=0; int ok=0, failed=0;
 for(int it=0;it<8;it++){ double y[4]={x[0],x[1],x[2],x[3]};
   double z1=y[1]-l10*y[0], z2=y[2]-l20*y[0]-l21*z1, z3=y[3]-l30*y[0]-l31*z1-l32*z2;
   y[3]=z3*r3; y[2]=z2*r2-l32*y[3]; y[1]=z1*r1-l21*y[2]-l31*y[3]; y[0]=y[0]*r0-l10*y[1]-l20*y[2]-l30*y[3];
   is=1/sqrt(y[0]*y[0]+y[1]*y[1]+y[2]*y[2]+y[3]*y[3]); dd=0; for(int q=0;q<4;q++){y[q]*=is; double e=y[q]-x[q]; dd+=e*e; x[q]=y[q];}
   int conv = dd<=1e-26 || (dd<=1e-16 && dd*dd<=1e-26*prev);
   if(it>=1){ if(conv){ok=1;break;} if(!(dd<0.25*prev)){failed=1;break;} } prev=dd; }
 for(int q=0;q<4;q++)nv[q]=x[q];
 float est = sqrtf((float)dd)*sqrtf((float)dd/fmaxf((float)dd,(float)prev));
 float trM = (float)(m[0][0]+m[1][1]+m[2][2]+m[3][3]);
 float f0=1.f/(float)D0, f1=1.f/(float)a11, f2=1.f/(float)b22, L10=l10, L20=l20, L21=l21; float q2 = L10*L21-L20;
 float trinv = f0*(1+L10*L10+q2*q2) + f1*(1+L21*L21) + f2;
 *delta = C1*est + C2*2.22e-16f*sqrtf(trM*trinv);
 return ok && !failed; }
int main(int argc, char**argv){ if(argc>1) NF32=atoi(argv[1]); if(argc>2) KAP=atof(argv[2]);
 FILE*f=fopen("/tmp/tri/sets.bin","rb"); int64_t ns; fread(&ns,8,1,f);
 for(int s=0;s<ns;s++){ int64_t n; fread(&n,8,1,f); double cp[80]; fread(cp,8,80,f); float* pts=malloc(n*16); fread(pts,16,n,f);
   long fbU=0, fbN=0, notok=0, mism=0, uncaught=0, umis=0, uncU=0;
   for(int64_t p=0;p<n;p++){ float ex[2],ey[2]; int certified=1;
     UD u[2]; float tx[2],ty[2];
     for(int v=0;v<2;v++){ const double* c=cp+40*v; double K[9]; for(int i=0;i<9;i++)K[i]=c[i];
        orc_undistort_points_f32(pts+p*4+v*2,1,K,c+9,5,&ex[v]); ey[v]=(&ex[v])[0]; /* placeholder */ }
     for(int v=0;v<2;v++){ const double* c=cp+40*v; double K[9]; float o[2]; for(int i=0;i<9;i++)K[i]=c[i];
        orc_undistort_points_f32(pts+p*4+v*2,1,K,c+9,5,o); ex[v]=o[0]; ey[v]=o[1];
        u[v]=undist_tol(pts[p*4+v*2],pts[p*4+v*2+1],c); tx[v]=(float)u[v].ox; ty[v]=(float)u[v].oy;
        int cu = dist_to_mid(u[v].ox)>2*u[v].delta && dist_to_mid(u[v].oy)>2*u[v].delta;
        int mu = tx[v]!=ex[v] || ty[v]!=ey[v]; if(mu) umis++; if(cu && mu) uncU++; if(!cu) certified=0; }
     if(!certified){ fbU++; continue; }
     /* exact path */
     double A[4][4], At[16], Vt[16];
     for(int v=0;v<2;v++){ const double* P=cp+40*v+26; for(int k=0;k<4;k++){ A[2*v][k]=(double)ex[v]*P[8+k]-P[k]; A[2*v+1][k]=(double)ey[v]*P[8+k]-P[4+k]; } }
     for(int c=0;c<4;c++)for(int r=0;r<4;r++)At[c*4+r]=A[r][c];
     orc_jacobi_svd(At,4,4,NULL,Vt);
     double B[4][4]; for(int v=0;v<2;v++){ const double* P=cp+40*v+26; for(int k=0;k<4;k++){ B[2*v][k]=fma((double)tx[v],P[8+k],-P[k]); B[2*v+1][k]=fma((double)ty[v],P[8+k],-P[4+k]); } }
     double nv[4], delta; int ok=null_tol(B,nv,&delta); if(!ok){notok++; continue;}
     int cn=1; for(int q=0;q<4;q++) if(!(dist_to_mid(nv[q])>2*delta)) cn=0;
     int mn=0; for(int q=0;q<4;q++){ float a=(float)Vt[12+q], b=(float)nv[q]; if(a!=b && a!=-b) mn=1; }
     /* sign: compare abs */
     if(mn) mism++; if(!cn) fbN++; if(cn&&mn) uncaught++;
   }
   printf("set %d n=%ld: undist fb %.2e (mism %ld uncaught %ld)  nv fb %.2e notok %.2e  nv mism %ld UNCAUGHT %ld\n", s, (long)n, fbU/(double)n, umis, uncU, fbN/(double)n, notok/(double)n, mism, uncaught);
   free(pts); }
}
