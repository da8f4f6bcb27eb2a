// FlowEvent.cpp — see FlowEvent.h (reference interface: /root/reference/src/FlowEvent.cpp:9-99).
#include "FlowEvent.h"

FlowEvent::FlowEvent(int x, int y, double t, int p, double Vx, double Vy)
    : x_(x), y_(y), pol_(p), t_(t), vx_(Vx), vy_(Vy), scale_(0) {}
FlowEvent::FlowEvent() : x_(0), y_(0), pol_(0), t_(0.0), vx_(0.0), vy_(0.0), scale_(0) {}

bool FlowEvent::setX(int v) { x_ = v; return true; }
bool FlowEvent::setY(int v) { y_ = v; return true; }
bool FlowEvent::setStamp(double v) { t_ = v; return true; }
bool FlowEvent::setPolarity(int v) { pol_ = v; return true; }
bool FlowEvent::setVx(double v) { vx_ = v; return true; }
bool FlowEvent::setVy(double v) { vy_ = v; return true; }
bool FlowEvent::setScale(int v) { scale_ = v; return true; }

int FlowEvent::getX() const { return x_; }
int FlowEvent::getY() const { return y_; }
double FlowEvent::getVx() const { return vx_; }
double FlowEvent::getVy() const { return vy_; }
double FlowEvent::getStamp() const { return t_; }
int FlowEvent::getPolarity() const { return pol_; }
int FlowEvent::getScale() const { return scale_; }
