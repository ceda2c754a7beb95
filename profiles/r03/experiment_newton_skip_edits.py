# Newton iterations (and zfacw, foedem): skip the exp / division whose weight is exactly 0
EDITS = [
    ("cloudsc_kcache.h", '''        real zqsat = (c.r2es * (a * exp_liq<real>(c, tt) + (R(1.0) - a) * exp_ice<real>(c, tt))) * zqp;''',
     '''        real el = R(0.0), ei = R(0.0);
        if (a != R(0.0)) el = exp_liq<real>(c, tt);
        if (a != R(1.0)) ei = exp_ice<real>(c, tt);
        real zqsat = (c.r2es * (a * el + (R(1.0) - a) * ei)) * zqp;'''),
    ("cloudsc_kcache.h", '''    { const real d = ztp1 - c.r4les; zfacw = cl_div(c.r5les, (d * d)); }''',
     '''    zfacw = R(0.0);
    if (zfoealfa != R(0.0)) { const real d = ztp1 - c.r4les; zfacw = cl_div(c.r5les, (d * d)); }'''),
    ("cloudsc_dev.h", '''  real dl = t - c.r4les, di = t - c.r4ies;
  return ((alfa * c.r5alvcp) * cl_div<real>(R(1.0), dl * dl)) + (((R(1.0) - alfa) * c.r5alscp) * cl_div<real>(R(1.0), di * di));''',
     '''  real tl = R(0.0), ti = R(0.0);
  if (alfa != R(0.0)) { const real dl = t - c.r4les; tl = (alfa * c.r5alvcp) * cl_div<real>(R(1.0), dl * dl); }
  if (alfa != R(1.0)) { const real di = t - c.r4ies; ti = ((R(1.0) - alfa) * c.r5alscp) * cl_div<real>(R(1.0), di * di); }
  return tl + ti;'''),
]
